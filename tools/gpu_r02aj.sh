#!/bin/bash
# Round-2 checkpoint: the GPU parity suite, then the profile + bench of
# profiles/run_profile.sh (kernel trace, FETCH_SIZE / WRITE_SIZE passes, bench).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02aj
export GKGPU_JIT_CACHE=$PWD/.jitcache
timeout -k 10 800 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r02aj/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r02aj/pytest.log
# assertion failures (rc 1) still allow the profile; crashes, aborts and time limits do not
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash profiles/run_profile.sh r02aj
