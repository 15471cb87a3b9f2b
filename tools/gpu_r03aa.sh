#!/bin/bash
# Join pass with multi-valued keys at HEAD: the join tests (verbose), then
# config 6 at 200K objects.   bash tools/gpu_r03aa.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03aa}
OUT=gpurun_out/$TAG
mkdir -p "$OUT" gpurun_out/jitcache
cp -n .jitcache/*.co gpurun_out/jitcache/ 2>/dev/null || true
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 600 python -u -m pytest tests/test_joins.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "join or unique or config6" > "$OUT/pytest_joins.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_joins.log"
if [ $rc -ne 0 ]; then echo JOINS_FAIL $rc; grep -E "FAILED|Error|assert" "$OUT/pytest_joins.log" | head -20; exit 1; fi
echo JOINS_OK
GKGPU_JOIN_TRACE=1 timeout -k 10 500 python -u bench.py --config 6 --pods 200000 --steps 10 --warmup 2 > "$OUT/c6_200k.json" 2> "$OUT/c6_200k.err" || { echo C6L_FAIL; tail "$OUT/c6_200k.err"; exit 1; }
echo C6_200K_OK
