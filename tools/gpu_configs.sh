#!/bin/bash
# Configs 3/4/5 at HEAD on one MI355X: config 5 batch and coalesced benches,
# then the rocprof trace + PMC + bench sequence (profiles/run_profile.sh) for
# configs 4 and 3.   bash tools/gpu_configs.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03c}
OUT=gpurun_out/$TAG
mkdir -p "$OUT" gpurun_out/jitcache
cp -n .jitcache/*.co gpurun_out/jitcache/ 2>/dev/null || true
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 300 python -u bench.py --config 5 --steps 1000 --warmup 20 > "$OUT/c5_batch.json" 2> "$OUT/c5_batch.err" || { echo C5_FAIL; tail "$OUT/c5_batch.err"; exit 1; }
echo C5_BATCH_OK
for rate in 20000 60000; do
  timeout -k 10 300 python -u bench.py --config 5 --steps 200 --warmup 20 --coalesce-us 300 --clients 64 --rate $rate --cpu-sample 0 > "$OUT/c5_coal_$rate.json" 2> "$OUT/c5_coal_$rate.err" || { echo C5C_FAIL; tail "$OUT/c5_coal_$rate.err"; exit 1; }
  echo C5_COAL_${rate}_OK
done
bash profiles/run_profile.sh ${TAG}_c4 --config 4 || { echo C4_PROFILE_FAIL; exit 1; }
echo C4_OK
bash profiles/run_profile.sh ${TAG}_c3 --config 3 || { echo C3_PROFILE_FAIL; exit 1; }
echo C3_OK
