#!/bin/bash
# GPU suite (-s: progress reaches the log) with the emit fast path's "{}"
# details fix and LDS lane scalars; then the LDS-scalar A/B on config 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02r
export GKGPU_JIT_CACHE=$PWD/.jitcache
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r02r/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r02r/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u tools/probe_repeat.py 1000000 $ONLY > gpurun_out/r02r/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/r02r/$tag.log; exit 1; }; echo "$tag: $(tail -1 gpurun_out/r02r/$tag.log)"; }
ONLY=""
run all_s0 GKGPU_LDS_SCALARS=0
run all_s1 X=1
exit $rc
