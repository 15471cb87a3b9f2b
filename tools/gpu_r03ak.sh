#!/bin/bash
# A/B of the early exit of constant-valued, error-free functions
(GKGPU_FN_EARLY=1 on), configs 2 and 4, alternating, then parity tests.
#   bash tools/gpu_r03ak.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03ak}
OUT=gpurun_out/$TAG
mkdir -p "$OUT" gpurun_out/jitcache
cp -n .jitcache/*.co gpurun_out/jitcache/ 2>/dev/null || true
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jitcache
run() {  # name cfg env...
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 400 python -u bench.py --config $cfg --steps 20 --warmup 3 --cpu-sample 0 > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "${name}_FAIL"; tail "$OUT/$name.err"; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); c = d["config"]
ks = {c["kernel_templates"].get(k["kernel"], k["kernel"])[:16]: round(k["avg_ms"], 3) for k in d["kernels"]}
print("AB", sys.argv[2], round(d["value"] / 1e6, 1), round(d["ms_per_step"], 3), ks)
PY
}
for rep in 1 2; do
  run c2_off_$rep 2 GKGPU_FN_EARLY=0 && run c2_on_$rep 2 GKGPU_FN_EARLY=1 && \
  run c4_off_$rep 4 GKGPU_FN_EARLY=0 && run c4_on_$rep 4 GKGPU_FN_EARLY=1 || exit 1
done
GKGPU_FN_EARLY=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_joins.py -m gpu -v --timeout 300 \
  --timeout-method thread -k "config2 or config4 or config6 or probes or limits or unique or join or scale or heavy or emission" > "$OUT/pytest.log" 2>&1
rc=$?
tail -2 "$OUT/pytest.log"
exit $rc
