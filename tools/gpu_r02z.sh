#!/bin/bash
# GPU suite with the JIT lookup CSE, then its A/B on config 2 (1M Pods).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02z
export GKGPU_JIT_CACHE=$PWD/.jitcache
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r02z/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r02z/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u tools/probe_repeat.py 1000000 > gpurun_out/r02z/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/r02z/$tag.log; exit 1; }; echo "$tag: $(tail -2 gpurun_out/r02z/$tag.log | head -1)"; }
run cse0 GKGPU_JIT_CSE=0
run cse1 X=1
exit $rc
