#!/bin/bash
# GPU: parity suite, then the bench on configs 2, 3 and 4 (one GPU each).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export GKGPU_JIT_CACHE=$PWD/.jitcache
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
echo PYTEST_OK; tail -2 gpurun_out/pytest_gpu.log
for c in 2 3 4; do
  timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 2 --cpu-sample 300 > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || { echo BENCH_FAIL $c; tail gpurun_out/bench_c$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/bench_c$c.json')); print('config $c value', round(d['value']/1e6,2), 'M evals/s ms/step', round(d['ms_per_step'],2), 'fb', d['config']['fallback_reviews'], 'err', d['config']['error_reviews'], 'cpu', round(d['cpu_baseline']['value'],1))
for k in d['kernels']: print('  ', d['config']['kernel_templates'].get(k['kernel'], k['kernel']), round(k['avg_ms'],3), k['constraints'], k['tuples'])"
done
