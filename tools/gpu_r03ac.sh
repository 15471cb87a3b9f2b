#!/bin/bash
# A/B of the fused multi-template kernel (GKGPU_FUSED=1) against the
# per-template kernels on configs 2 and 4, then the fused kernel's parity on
# config 2 and config 4 tests.  A ticker keeps the call's output alive while
# hipRTC compiles a fused kernel that is not in the cache (minutes).
#   bash tools/gpu_r03ac.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03ac}
OUT=gpurun_out/$TAG
mkdir -p "$OUT" gpurun_out/jitcache
cp -n .jitcache/*.co gpurun_out/jitcache/ 2>/dev/null || true
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jitcache
( while true; do echo "tick $(date +%T)" >> "$OUT/ticker.log"; sleep 30; done ) &
TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
for cfg in 2 4; do
  for f in 0 1; do
    GKGPU_FUSED=$f timeout -k 10 500 python -u bench.py --config $cfg --steps 20 --warmup 3 --cpu-sample 0 > "$OUT/c${cfg}_f$f.json" 2> "$OUT/c${cfg}_f$f.err" || { echo "C${cfg}_F${f}_FAIL"; tail "$OUT/c${cfg}_f$f.err"; exit 1; }
    echo "C${cfg}_F${f}_OK $(python -c "import json;d=json.load(open('$OUT/c${cfg}_f$f.json'));print(round(d['value']/1e6,1), round(d['ms_per_step'],3))")"
  done
done
GKGPU_FUSED=1 timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 600 --timeout-method thread \
  -k "config2_agilebank_pods or config4_mixed" > "$OUT/pytest_fused.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_fused.log"
exit $rc
