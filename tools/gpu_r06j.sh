#!/bin/bash
# Round-6 HEAD: configs 3/4/6/5/5-coalesced/from-cache with their CPU
# baselines (tools/gpu_final.sh part b), then a config-2 probe: the template
# kernels with their emission sites cut out (GKGPU_JIT_PATCH; rows differ, the
# time is what the emission path costs) and the passes' grid at capacity
# (GKGPU_PASS_HINT=0).
#   bash tools/gpu_r06j.sh <tag>
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r06j}
bash tools/gpu_final.sh "$TAG" b || exit 1
bash tools/gpu_bench_ab.sh ${TAG}_probe "--steps 20 --warmup 3 --shard-leg off --cpu-e2e off" "" \
  "GKGPU_JIT_PATCH=@tools/probes/noemit_args.txt" "GKGPU_PASS_HINT=0" || exit 1
mkdir -p gpurun_out/$TAG
GKGPU_FLATTEN_TRACE=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 --shard-leg off --cpu-e2e off > gpurun_out/$TAG/trace.json 2> gpurun_out/$TAG/trace.err || { echo TRACE_FAIL; exit 1; }
grep -E "^(sync strings|stage upload|flatten: (parse|intern))" gpurun_out/$TAG/trace.err
