#!/bin/bash
# GPU suite after the format-pass change, then config 2 kernel times.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02ak
export GKGPU_JIT_CACHE=$PWD/.jitcache
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r02ak/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r02ak/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/probe_repeat.py 1000000 > gpurun_out/r02ak/all.log 2>&1 || { tail -5 gpurun_out/r02ak/all.log; exit 1; }
tail -2 gpurun_out/r02ak/all.log
exit $rc
