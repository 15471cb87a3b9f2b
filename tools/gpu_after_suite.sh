#!/bin/bash
# GPU diagnostic: is the bench slower after the GPU test suite because of the
# on-disk JIT cache or because of the GPU's state?  A: bench; pytest; B: bench
# (same cache); C: bench with a fresh cache.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export GKGPU_JIT_CACHE=$PWD/.jitcache
b() { timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/as_$1.json 2>gpurun_out/as_$1.err && python3 -c "
import json; d=json.load(open('gpurun_out/as_$1.json')); print('$1', round(d['value']/1e6,1), round(d['ms_per_step'],2), [(k['kernel'][-6:], round(k['avg_ms'],2)) for k in d['kernels']])"; }
b A || exit 1
ls -la .jitcache > gpurun_out/as_cache_before.txt 2>&1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_as.log 2>&1 || { echo PYTEST_FAIL; tail -20 gpurun_out/pytest_as.log; exit 1; }
ls -la .jitcache > gpurun_out/as_cache_after.txt 2>&1
b B || exit 1
GKGPU_JIT_CACHE=/tmp/gk_fresh_cache b C || exit 1
b D
