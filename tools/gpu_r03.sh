#!/bin/bash
# Round-3 GPU check: the parity suite (verbose log, per-test timeout), then a
# short default bench.  Usage (on the GPU box, from the repo root):
#   bash tools/gpu_r03.sh <tag> [pytest -k expression]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
# template-kernel code objects: start from the tree's .jitcache, collect new
# ones under gpurun_out/ (merged back; copy them into .jitcache afterwards)
mkdir -p gpurun_out/jitcache
cp -n .jitcache/*.co gpurun_out/jitcache/ 2>/dev/null || true
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jitcache
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > "$OUT/pytest_gpu.log" 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
fi
rc=$?
tail -5 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ]; then echo PYTEST_FAIL $rc; grep -E "FAILED|Error|error" "$OUT/pytest_gpu.log" | head -20; exit 1; fi
echo PYTEST_OK
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --cpu-sample 200000 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo BENCH_FAIL; tail "$OUT/bench.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); print('value', d['value'], 'ms/step', d['ms_per_step'], 'frac', d['roofline']['frac'])
for k in d['kernels']: print(k)"
