#!/bin/bash
# Inventory join indexes on one MI355X: the join tests first (verbose), then
# the whole -m gpu suite, then config 6 benches (20K and 200K objects; the
# 20K one also with GKGPU_JOINS=0, the scan).
#   bash tools/gpu_r03y.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03y}
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
timeout -k 10 400 python -u bench.py --config 6 --steps 5 --warmup 1 --cpu-sample 0 > "$OUT/c6_20k.json" 2> "$OUT/c6_20k.err" || { echo C6_FAIL; tail "$OUT/c6_20k.err"; exit 1; }
echo C6_20K_OK
GKGPU_JOINS=0 timeout -k 10 400 python -u bench.py --config 6 --steps 3 --warmup 1 --cpu-sample 0 > "$OUT/c6_20k_scan.json" 2> "$OUT/c6_20k_scan.err" || { echo C6S_FAIL; tail "$OUT/c6_20k_scan.err"; exit 1; }
echo C6_20K_SCAN_OK
timeout -k 10 500 python -u bench.py --config 6 --pods 200000 --steps 5 --warmup 1 --cpu-sample 0 > "$OUT/c6_200k.json" 2> "$OUT/c6_200k.err" || { echo C6L_FAIL; tail "$OUT/c6_200k.err"; exit 1; }
echo C6_200K_OK
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  --deselect tests/test_joins.py > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ]; then echo PYTEST_FAIL $rc; grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20; exit 1; fi
echo PYTEST_OK
