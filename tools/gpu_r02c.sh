#!/bin/bash
# A/B of the hot-builtin inlining (GKGPU_INLINE_HOT) on K8sContainerLimits and
# the whole config 2, then the GPU parity suite on the default build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02c
export GKGPU_JIT_CACHE=$PWD/.jitcache
run() { GKGPU_INLINE_HOT=$2 timeout -k 10 240 python -u tools/probe_repeat.py 1000000 $3 > gpurun_out/r02c/$1.log 2>&1 || { echo "FAIL $1"; tail -5 gpurun_out/r02c/$1.log; exit 1; }; echo "$1: $(tail -1 gpurun_out/r02c/$1.log)"; }
run cl_h0 0 K8sContainerLimits
run cl_h1 1 K8sContainerLimits
run all_h0 0 ""
run all_h1 1 ""
run cl_h1b 1 K8sContainerLimits
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02c/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r02c/pytest.log
exit $rc
