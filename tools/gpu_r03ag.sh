#!/bin/bash
# A clean JIT cache for the round-end run: smoke(), the whole -m gpu suite and
# the default bench with an EMPTY cache directory, so every code object under
# gpurun_out/jc_clean/ is one the current runtime compiled (then copied into
# .jitcache/ by hand).   bash tools/gpu_r03ag.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03ag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT" gpurun_out/jc_clean
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jc_clean
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo SMOKE_FAIL; tail "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -2 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ]; then echo PYTEST_FAIL $rc; grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20; exit 1; fi
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo BENCH_FAIL; tail "$OUT/bench.err"; exit 1; }
echo BENCH_OK
