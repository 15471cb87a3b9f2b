#!/bin/bash
# Configs 3, 4, 5 (batch) and 6 (200K) benches at HEAD, one call.
#   bash tools/gpu_r03aj.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03aj}
OUT=gpurun_out/$TAG
mkdir -p "$OUT" gpurun_out/jitcache
cp -n .jitcache/*.co gpurun_out/jitcache/ 2>/dev/null || true
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 400 python -u bench.py --config 3 > "$OUT/c3.json" 2> "$OUT/c3.err" || { echo C3_FAIL; tail "$OUT/c3.err"; exit 1; }
echo C3_OK
timeout -k 10 400 python -u bench.py --config 4 > "$OUT/c4.json" 2> "$OUT/c4.err" || { echo C4_FAIL; tail "$OUT/c4.err"; exit 1; }
echo C4_OK
timeout -k 10 300 python -u bench.py --config 5 --steps 1000 --warmup 20 > "$OUT/c5.json" 2> "$OUT/c5.err" || { echo C5_FAIL; tail "$OUT/c5.err"; exit 1; }
echo C5_OK
timeout -k 10 500 python -u bench.py --config 6 --pods 200000 > "$OUT/c6_200k.json" 2> "$OUT/c6_200k.err" || { echo C6_FAIL; tail "$OUT/c6_200k.err"; exit 1; }
echo C6_OK
