#!/bin/bash
# A/B in one call: the inlined emission fast path (GK_EMIT_FAST, deferred
# sizing in finish_lane) on K8sRequiredProbes, K8sContainerLimits and all of
# config 2 (inline set add / set difference in both legs); then the GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02o
export GKGPU_JIT_CACHE=$PWD/.jitcache
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u tools/probe_repeat.py 1000000 $ONLY > gpurun_out/r02o/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/r02o/$tag.log; exit 1; }; echo "$tag: $(tail -2 gpurun_out/r02o/$tag.log | tr '\n' ' ')"; }
ONLY=K8sRequiredProbes
run rp_ef0 GKGPU_JIT_PRE=GK_EMIT_FAST=0
run rp_ef1 X=1
ONLY=K8sContainerLimits
run cl_ef0 GKGPU_JIT_PRE=GK_EMIT_FAST=0
run cl_ef1 X=1
ONLY=""
run all_ef1 X=1
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r02o/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r02o/pytest.log
exit $rc
