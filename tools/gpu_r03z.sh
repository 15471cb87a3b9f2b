#!/bin/bash
# Round-3 join pass at HEAD on one MI355X: the whole -m gpu suite, the
# default bench (config 2), then config 6 at 20K and 200K objects.
#   bash tools/gpu_r03z.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03z}
OUT=gpurun_out/$TAG
mkdir -p "$OUT" gpurun_out/jitcache
cp -n .jitcache/*.co gpurun_out/jitcache/ 2>/dev/null || true
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ]; then echo PYTEST_FAIL $rc; grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20; exit 1; fi
echo PYTEST_OK
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > "$OUT/c2.json" 2> "$OUT/c2.err" || { echo C2_FAIL; tail "$OUT/c2.err"; exit 1; }
echo C2_OK
timeout -k 10 400 python -u bench.py --config 6 --steps 20 --warmup 3 > "$OUT/c6_20k.json" 2> "$OUT/c6_20k.err" || { echo C6_FAIL; tail "$OUT/c6_20k.err"; exit 1; }
echo C6_20K_OK
GKGPU_JOIN_TRACE=1 timeout -k 10 500 python -u bench.py --config 6 --pods 200000 --steps 10 --warmup 2 > "$OUT/c6_200k.json" 2> "$OUT/c6_200k.err" || { echo C6L_FAIL; tail "$OUT/c6_200k.err"; exit 1; }
echo C6_200K_OK
