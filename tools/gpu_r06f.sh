#!/bin/bash
# Round-6: the column directory in LDS (devrt.h GK_CV_LDS) -- GPU suite at the
# new default, then A/B against GKGPU_CV_LDS=0 and 3 waves per EU on configs 2, 4.
#   bash tools/gpu_r06f.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r06f}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export GKGPU_JIT_CACHE=/tmp/gkjit_cache
mkdir -p $GKGPU_JIT_CACHE && cp -n .jitcache/*.co $GKGPU_JIT_CACHE/ 2>/dev/null
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc = 0 ] || exit 1
bash tools/gpu_bench_ab.sh ${TAG}_c2 "--steps 20 --warmup 3 --shard-leg off --cpu-e2e off" "" "GKGPU_CV_LDS=0" "GKGPU_JIT_WPE=3" "" || exit 1
bash tools/gpu_bench_ab.sh ${TAG}_c4 "--config 4 --steps 10 --warmup 2 --cpu-e2e off" "" "GKGPU_CV_LDS=0" "GKGPU_JIT_WPE=3" || exit 1
