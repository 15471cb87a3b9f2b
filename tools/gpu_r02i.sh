#!/bin/bash
# Shared lookups in fused groups (GKGPU_FUSE_CSE) and top-level violation-body
# fusion: order/parity tests, then an A/B on K8sContainerLimits and config 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02i
export GKGPU_JIT_CACHE=$PWD/.jitcache
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -v --timeout 200 --timeout-method thread \
  -k "emission_order or config2 or audit_writer or libs or config4 or integration" > gpurun_out/r02i/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r02i/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
run() { local tag=$1; shift; env "$@" timeout -k 10 240 python -u tools/probe_repeat.py 1000000 $ONLY > gpurun_out/r02i/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/r02i/$tag.log; exit 1; }; echo "$tag: $(tail -1 gpurun_out/r02i/$tag.log)"; }
ONLY=K8sContainerLimits
run cl_cse0 GKGPU_FUSE_CSE=0
run cl_cse1 X=1
run cl_cse0b GKGPU_FUSE_CSE=0
run cl_cse1b X=1
ONLY=""
run all_cse1 X=1
exit $rc
