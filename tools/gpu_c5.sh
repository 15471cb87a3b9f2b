#!/bin/bash
# GPU: config-5 webhook parity test, then the config-5 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export GKGPU_JIT_CACHE=$PWD/.jitcache
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "config5 or string_builtins" -x -q --timeout 250 --timeout-method thread > gpurun_out/pytest_c5.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_c5.log; exit 1; }
echo PYTEST_OK; tail -2 gpurun_out/pytest_c5.log
timeout -k 10 300 python -u bench.py --config 5 --warmup 20 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo BENCH_FAIL; tail gpurun_out/bench_c5.err; exit 1; }
cat gpurun_out/bench_c5.json
