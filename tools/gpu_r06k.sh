#!/bin/bash
# Round-6: format-pass literals copied a dword at a time (kernels.hip
# LOut::put_lit) -- GPU suite, then config-2 A/B against the library built
# without it (tools/ab/libgkgpu_base.so), alternating.
#   bash tools/gpu_r06k.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r06k}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export GKGPU_JIT_CACHE=/tmp/gkjit_cache
mkdir -p $GKGPU_JIT_CACHE && cp -n .jitcache/*.co $GKGPU_JIT_CACHE/ 2>/dev/null
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc = 0 ] || exit 1
bash tools/gpu_bench_ab.sh ${TAG}_ab "--steps 20 --warmup 3 --shard-leg off --cpu-e2e off" "" "GKGPU_LIB=tools/ab/libgkgpu_base.so" "" \
  "GKGPU_LIB=tools/ab/libgkgpu_base.so" || exit 1
