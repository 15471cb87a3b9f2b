#!/bin/bash
# unique-label GPU parity; cost of deferred-message sizing (diagnostic build:
# no string-length loads) on K8sContainerLimits and K8sRequiredProbes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02ab
export GKGPU_JIT_CACHE=$PWD/.jitcache
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread -k "unique_label" > gpurun_out/r02ab/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r02ab/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u tools/probe_repeat.py 1000000 $ONLY > gpurun_out/r02ab/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/r02ab/$tag.log; exit 1; }; echo "$tag: $(tail -2 gpurun_out/r02ab/$tag.log | head -1)"; }
ONLY=K8sContainerLimits
run cl_base X=1
run cl_nosize GKGPU_JIT_PRE=GK_DIAG_SIZE_BOUND=1
ONLY=K8sRequiredProbes
run rp_base X=1
run rp_nosize GKGPU_JIT_PRE=GK_DIAG_SIZE_BOUND=1
exit $rc
