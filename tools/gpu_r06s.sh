#!/bin/bash
# Round-6 final: small programs at 4 waves unless they iterate a parameter
# collection inside another loop over parameters or use regular expressions
# (jit.cc wpe_of) -- GPU suite, then configs 2 and 4 against the 3-wave rule
# (GKGPU_JIT_WPE does not separate them: the old rule is reproduced by the
# numbers of r06r's default runs on the same HEAD otherwise).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r06s}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export GKGPU_JIT_CACHE=/tmp/gkjit_cache
mkdir -p $GKGPU_JIT_CACHE && cp -n .jitcache/*.co $GKGPU_JIT_CACHE/ 2>/dev/null
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc = 0 ] || exit 1
bash tools/gpu_bench_ab.sh ${TAG}_ab "--steps 20 --warmup 3 --shard-leg off --cpu-e2e off" "" "" || exit 1
bash tools/gpu_bench_ab.sh ${TAG}_c4 "--config 4 --steps 10 --warmup 2 --cpu-e2e off" "" || exit 1
