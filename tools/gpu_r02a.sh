#!/bin/bash
# Round-2 checkpoint: GPU parity suite, then a short config-2 bench (5 constraints).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export GKGPU_JIT_CACHE=$PWD/.jitcache
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02a_pytest.log 2>&1; rc=$?
tail -5 gpurun_out/r02a_pytest.log
[ $rc = 0 ] || { grep -E "FAILED|Error|error" gpurun_out/r02a_pytest.log | head -20; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-sample 200 > gpurun_out/r02a_bench.json 2> gpurun_out/r02a_bench.err || { tail -20 gpurun_out/r02a_bench.err; exit 1; }
cat gpurun_out/r02a_bench.json
