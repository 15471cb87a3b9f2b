#!/bin/bash
# Round-6 probe of the lane heap in the set-building templates (config 4's
# K8sRequiredLabels): list headers sized for one element (lists grow by
# relocation, tools/probes/list_cap_small.txt) so more lists stay in the LDS
# heap words, and 24 LDS heap words; configs 4 and 2, per-kernel times.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r06p}
export GKGPU_JIT_CACHE=/tmp/gkjit_cache
mkdir -p $GKGPU_JIT_CACHE && cp -n .jitcache/*.co $GKGPU_JIT_CACHE/ 2>/dev/null
bash tools/gpu_bench_ab.sh ${TAG}_c4 "--config 4 --steps 10 --warmup 2 --cpu-e2e off" "" "GKGPU_JIT_PATCH=@tools/probes/list_cap_small.txt" "GKGPU_LDS_HEAP=24" || exit 1
bash tools/gpu_bench_ab.sh ${TAG}_c2 "--steps 20 --warmup 3 --shard-leg off --cpu-e2e off" "" "GKGPU_JIT_PATCH=@tools/probes/list_cap_small.txt" "GKGPU_LDS_HEAP=24" || exit 1
