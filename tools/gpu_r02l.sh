#!/bin/bash
# K8sRequiredProbes message-path variants, and the device's CU count / clock.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02l
export GKGPU_JIT_CACHE=$PWD/.jitcache
timeout -k 10 240 python -u tools/probe_repeat.py 1000000 > gpurun_out/r02l/all.log 2>&1 || { tail -5 gpurun_out/r02l/all.log; exit 1; }
tail -2 gpurun_out/r02l/all.log
timeout -k 10 600 python -u tools/probe_variants_rp.py 1000000 full,const_msg,inline_msg,one_arg_msg,const_args_msg > gpurun_out/r02l/rp_variants.log 2>&1 || { tail -5 gpurun_out/r02l/rp_variants.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r02l/rp_variants.log
