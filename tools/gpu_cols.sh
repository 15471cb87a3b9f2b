#!/bin/bash
# Column-form staged batches on one MI355X: a small parity check first, then
# the GPU suite and the config-2 / config-4 bench with the column form
# (GKGPU_COLUMNS=1), and the node form beside it (A/B, same box).
#   bash tools/gpu_cols.sh <tag> [suite]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; SUITE=${2:-suite}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
JC=/tmp/gkjit_cache
mkdir -p "$JC"
cp -n .jitcache/*.co "$JC/" 2>/dev/null || true
export GKGPU_JIT_CACHE=$JC
jit_pull() {
  local new=() f sz=0
  for f in "$JC"/*.co; do [ -e ".jitcache/$(basename "$f")" ] || { new+=("$f"); sz=$((sz + $(stat -c %s "$f"))); }; done
  if [ ${#new[@]} -gt 0 ] && [ $sz -lt 40000000 ]; then mkdir -p gpurun_out/jitcache_new && cp -n "${new[@]}" gpurun_out/jitcache_new/; fi
  echo "jit cache: ${#new[@]} new code objects, $sz bytes"
}
trap jit_pull EXIT
export GKGPU_COLUMNS=1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -2 "$OUT/smoke.log"; [ $rc = 0 ] || exit 1
if [ "$SUITE" = suite ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc = 0 ] || exit 1
fi
for c in 2 4; do
  for v in 1 0; do
    GKGPU_COLUMNS=$v timeout -k 10 400 python -u bench.py --config $c --cpu-sample 0 > "$OUT/c${c}_cols$v.json" 2> "$OUT/c${c}_cols$v.err" || { echo "BENCH_FAIL c$c cols$v"; tail "$OUT/c${c}_cols$v.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('C'+sys.argv[2], 'cols', sys.argv[3], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms; e2e', round(c.get('end_to_end_evals_per_s',0)/1e6,1), 'M/s; upload', c.get('upload_bytes_per_resource'), 'B/res; stage', c.get('stage_s'))" "$OUT/c${c}_cols$v.json" $c $v
  done
done
