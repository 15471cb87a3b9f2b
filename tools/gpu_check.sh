#!/bin/bash
# GPU check after a change: parity suite, then the default bench (short).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export GKGPU_JIT_CACHE=$PWD/.jitcache
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
echo PYTEST_OK
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --cpu-sample 300 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail gpurun_out/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench.json')); print('value', d['value'], 'ms/step', d['ms_per_step'])
for k in d['kernels']: print(k)"
