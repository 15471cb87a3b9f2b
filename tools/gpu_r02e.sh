#!/bin/bash
# Cost breakdown of the K8sContainerLimits predicate by template variants
# (tools/probe_variants.py), with the GPU clocks sampled around it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02e
export GKGPU_JIT_CACHE=$PWD/.jitcache
rocm-smi --showclocks > gpurun_out/r02e/clocks_before.txt 2>&1 || true
timeout -k 10 900 python -u tools/probe_variants.py 1000000 > gpurun_out/r02e/variants.log 2>&1; rc=$?
rocm-smi --showclocks > gpurun_out/r02e/clocks_after.txt 2>&1 || true
cat gpurun_out/r02e/variants.log | tail -12
exit $rc
