#!/bin/bash
# A/B in one call: lane-constant input paths (GKGPU_LANE_PATHS) and the LDS
# lane heap (GKGPU_LDS_HEAP) on K8sRequiredProbes, K8sContainerLimits and all of
# config 2; then parity tests with the LDS heap on.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02m
export GKGPU_JIT_CACHE=$PWD/.jitcache
run() { local tag=$1; shift; env "$@" timeout -k 10 240 python -u tools/probe_repeat.py 1000000 $ONLY > gpurun_out/r02m/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/r02m/$tag.log; exit 1; }; echo "$tag: $(tail -2 gpurun_out/r02m/$tag.log | tr '\n' ' ')"; }
ONLY=K8sRequiredProbes
run rp_lp0 GKGPU_LANE_PATHS=0
run rp_lp1 X=1
run rp_lds16 GKGPU_LDS_HEAP=16
run rp_lds32 GKGPU_LDS_HEAP=32
ONLY=K8sContainerLimits
run cl_lp0 GKGPU_LANE_PATHS=0
run cl_lp1 X=1
run cl_lds16 GKGPU_LDS_HEAP=16
run cl_lds32 GKGPU_LDS_HEAP=32
ONLY=""
run all_lp0 GKGPU_LANE_PATHS=0
run all_lp1 X=1
run all_lds32 GKGPU_LDS_HEAP=32
GKGPU_LDS_HEAP=32 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -v --timeout 200 --timeout-method thread \
  -k "emission_order or config2 or config5 or audit_writer or libs or config4_mixed or string_builtins" > gpurun_out/r02m/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r02m/pytest.log
exit $rc
