#!/bin/bash
# Round-6 occupancy grid: waves per EU x LDS heap words for every template at
# once (each kernel's time is read off its own line), configs 2 and 4.
#   bash tools/gpu_r06g.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r06g}
export GKGPU_JIT_CACHE=/tmp/gkjit_cache
mkdir -p $GKGPU_JIT_CACHE && cp -n .jitcache/*.co $GKGPU_JIT_CACHE/ 2>/dev/null
S=("" "GKGPU_JIT_WPE=3" "GKGPU_JIT_WPE=4 GKGPU_LDS_HEAP=8" "GKGPU_JIT_WPE=3 GKGPU_LDS_HEAP=8" "GKGPU_JIT_WPE=2" \
   "GKGPU_JIT_WPE=4 GKGPU_LDS_HEAP=12" "GKGPU_JIT_WPE=4 GKGPU_LDS_HEAP=4")
bash tools/gpu_bench_ab.sh ${TAG}_c2 "--steps 20 --warmup 3 --shard-leg off --cpu-e2e off" "${S[@]}" || exit 1
bash tools/gpu_bench_ab.sh ${TAG}_c4 "--config 4 --steps 10 --warmup 2 --cpu-e2e off" "${S[@]}" || exit 1
