cd "$GRAFT_REPO_ROOT"
TAG=${1:-r05t}
mkdir -p gpurun_out/$TAG /tmp/gkjit_cache; cp -n .jitcache/*.co /tmp/gkjit_cache/ 2>/dev/null; export GKGPU_JIT_CACHE=/tmp/gkjit_cache
i=0
for v in ${DIAG_VARIANTS:-"GKGPU_GMEMO=1"}; do
  i=$((i+1))
  env $v timeout -k 10 300 python -u tools/diag_rows.py > gpurun_out/$TAG/v$i.log 2>&1; rc=$?
  echo "[$v] rc $rc $(grep -E '^(rows|flagged)' gpurun_out/$TAG/v$i.log | tr '\n' ' ')"
  [ $rc = 0 ] || exit 1
done
