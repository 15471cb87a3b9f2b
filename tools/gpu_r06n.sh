#!/bin/bash
# Round-6: launch-bound waves apart from the LDS plan (jit.cc GKGPU_JIT_LB):
# every template's kernel at 4 and at 3 waves per EU in its launch bounds while
# its LDS stage keeps the default plan; configs 2 and 4, per-kernel times.
#   bash tools/gpu_r06n.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r06n}
export GKGPU_JIT_CACHE=/tmp/gkjit_cache
mkdir -p $GKGPU_JIT_CACHE && cp -n .jitcache/*.co $GKGPU_JIT_CACHE/ 2>/dev/null
bash tools/gpu_bench_ab.sh ${TAG}_c2 "--steps 20 --warmup 3 --shard-leg off --cpu-e2e off" "" "GKGPU_JIT_LB=4" "GKGPU_JIT_LB=3" "" || exit 1
bash tools/gpu_bench_ab.sh ${TAG}_c4 "--config 4 --steps 10 --warmup 2 --cpu-e2e off" "" "GKGPU_JIT_LB=4" "GKGPU_JIT_LB=3" || exit 1
