#!/bin/bash
# Clock probe + K8sRequiredProbes cost breakdown by template variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02k
export GKGPU_JIT_CACHE=$PWD/.jitcache
timeout -k 10 240 python -u tools/probe_repeat.py 1000000 > gpurun_out/r02k/all.log 2>&1 || { tail -5 gpurun_out/r02k/all.log; exit 1; }
tail -2 gpurun_out/r02k/all.log
timeout -k 10 600 python -u tools/probe_variants_rp.py 1000000 > gpurun_out/r02k/rp_variants.log 2>&1 || { tail -5 gpurun_out/r02k/rp_variants.log; exit 1; }
cat gpurun_out/r02k/rp_variants.log
run() { local tag=$1; shift; env "$@" timeout -k 10 240 python -u tools/probe_repeat.py 1000000 $ONLY > gpurun_out/r02k/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/r02k/$tag.log; exit 1; }; echo "$tag: $(tail -2 gpurun_out/r02k/$tag.log | tr '\n' ' ')"; }
ONLY=K8sRequiredProbes
run rp_lv1 GKGPU_MEMO_LOOPVAR=1
run rp_lv0 X=1
run rp_lv1b GKGPU_MEMO_LOOPVAR=1
run rp_lv0b X=1
