#!/bin/bash
# Rule-body fusion (GKGPU_FUSE): the order/parity tests that cover it, then an
# A/B of K8sContainerLimits and of config 2 in one call (alternating).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02g
export GKGPU_JIT_CACHE=$PWD/.jitcache
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -v --timeout 200 --timeout-method thread \
  -k "emission_order or config2 or audit_writer or container or libs" > gpurun_out/r02g/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r02g/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
run() { GKGPU_FUSE=$2 timeout -k 10 240 python -u tools/probe_repeat.py 1000000 $3 > gpurun_out/r02g/$1.log 2>&1 || { echo "FAIL $1"; tail -5 gpurun_out/r02g/$1.log; exit 1; }; echo "$1: $(tail -1 gpurun_out/r02g/$1.log)"; }
run cl_f0 0 K8sContainerLimits
run cl_f1 1 K8sContainerLimits
run all_f0 0 ""
run all_f1 1 ""
run cl_f1b 1 K8sContainerLimits
exit $rc
