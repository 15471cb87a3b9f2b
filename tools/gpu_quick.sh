#!/bin/bash
# Quick GPU check after a device-runtime change: K8sContainerLimits kernel time
# at 1M Pods, then the template kernel vs the bytecode VM on 200k Pods.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export GKGPU_JIT_CACHE=0
timeout -k 10 150 python -u tools/probe_repeat.py 1000000 ${1:-K8sContainerLimits} > gpurun_out/quick_time.log 2>&1 || { echo TIME_FAIL; tail -20 gpurun_out/quick_time.log; exit 1; }
tail -3 gpurun_out/quick_time.log
timeout -k 10 300 python -u tools/probe_diff.py 200000 ${1:-K8sContainerLimits} '[["jit", {}]]' > gpurun_out/quick_diff.log 2>&1 || { echo DIFF_FAIL; tail -20 gpurun_out/quick_diff.log; exit 1; }
cat gpurun_out/quick_diff.log
