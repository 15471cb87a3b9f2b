#!/bin/bash
# coalescer diagnostics + config-4 flagged-review A/B (memo strings / memo node keys / path layout)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03p
mkdir -p "$OUT" gpurun_out/jitcache
cp -n .jitcache/*.co gpurun_out/jitcache/ 2>/dev/null || true
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 300 python -u -m pytest tests/test_coalescer.py -m gpu -v -s --timeout 240 --timeout-method thread > $OUT/coal.log 2>&1
rc=$?; tail -3 $OUT/coal.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
for v in "" GKGPU_MEMO_STRINGS=0 GKGPU_MEMO_NODES=0 GKGPU_PATH_LAYOUT=0; do
  echo "== $v"
  env $v timeout -k 10 240 python -u tools/probe_flags.py 4 1250000 > "$OUT/flags_${v:-default}.log" 2>&1 || { echo PROBE_FAIL; tail -5 "$OUT/flags_${v:-default}.log"; exit 1; }
  grep -E "flagged|reasons|kinds" "$OUT/flags_${v:-default}.log"
done
