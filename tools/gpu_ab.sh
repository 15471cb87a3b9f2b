#!/bin/bash
# GPU diagnostic: bench before and after the GPU test suite in one call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export GKGPU_JIT_CACHE=$PWD/.jitcache
b() { timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/ab_$1.json 2>gpurun_out/ab_$1.err && python3 -c "
import json; d=json.load(open('gpurun_out/ab_$1.json')); print('$1', round(d['ms_per_step'],2), [(k['kernel'][-6:], round(k['avg_ms'],2)) for k in d['kernels']])"; }
b A || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
echo PYTEST_OK
b B || exit 1
rocm-smi --showclocks --showtemp --showpower 2>&1 | tail -20 > gpurun_out/smi.txt
b C
