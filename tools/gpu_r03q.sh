#!/bin/bash
# coalescer test after the context node-buffer fix + config-4 repeated sweeps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03q
mkdir -p "$OUT" gpurun_out/jitcache
cp -n .jitcache/*.co gpurun_out/jitcache/ 2>/dev/null || true
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 300 python -u -m pytest tests/test_coalescer.py tests/test_concurrency.py -m gpu -v -s --timeout 240 --timeout-method thread > $OUT/coal.log 2>&1
rc=$?; tail -3 $OUT/coal.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
timeout -k 10 300 python -u tools/probe_flags.py 4 1250000 > "$OUT/flags.log" 2>&1 || { echo PROBE_FAIL; tail -5 "$OUT/flags.log"; exit 1; }
grep -E "sweep|flagged|reasons|kinds" "$OUT/flags.log"
