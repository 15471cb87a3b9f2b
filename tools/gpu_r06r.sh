#!/bin/bash
# Round-6 re-check of two JIT switches under the column form: outlined
# memo-miss bodies (GKGPU_JIT_OUTLINE=0 inlines them) and the per-wave LDS
# memo cache size (GKGPU_JIT_LDSMEMO=16 / 64; default 32); configs 2 and 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r06r}
export GKGPU_JIT_CACHE=/tmp/gkjit_cache
mkdir -p $GKGPU_JIT_CACHE && cp -n .jitcache/*.co $GKGPU_JIT_CACHE/ 2>/dev/null
S=("" "GKGPU_JIT_OUTLINE=0" "GKGPU_JIT_LDSMEMO=64" "GKGPU_JIT_LDSMEMO=16")
bash tools/gpu_bench_ab.sh ${TAG}_c2 "--steps 20 --warmup 3 --shard-leg off --cpu-e2e off" "${S[@]}" || exit 1
bash tools/gpu_bench_ab.sh ${TAG}_c4 "--config 4 --steps 10 --warmup 2 --cpu-e2e off" "${S[@]}" || exit 1
