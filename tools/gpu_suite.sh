#!/bin/bash
# GPU check: selected "first" tests (verbose, allowed to fail: their log is kept),
# then the whole -m gpu suite without them, then optionally the profile sequence
# of profiles/run_profile.sh.
#   bash tools/gpu_suite.sh <tag> <profile-tag|bench|-> [first test node ids...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; PROF=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
# (gpu_measure.sh / gpu_final.sh set GKGPU_JIT_CACHE; standalone: seeded from .jitcache)
if [ -z "$GKGPU_JIT_CACHE" ]; then mkdir -p /tmp/gkjit_cache; cp -n .jitcache/*.co /tmp/gkjit_cache/ 2>/dev/null || true; export GKGPU_JIT_CACHE=/tmp/gkjit_cache; fi
DESEL=()
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -v -s --timeout 300 --timeout-method thread > "$OUT/pytest_first.log" 2>&1
  rc=$?
  tail -3 "$OUT/pytest_first.log"
  # only test failures (rc 1) let the call go on; a timeout / crash ends it
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo FIRST_ABORT $rc; exit 1; fi
  for t in "$@"; do DESEL+=(--deselect "$t"); done
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${DESEL[@]}" > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ]; then echo PYTEST_FAIL $rc; grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20; exit 1; fi
echo PYTEST_OK
if [ "$PROF" = "bench" ]; then
  timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --cpu-sample 200000 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo BENCH_FAIL; tail "$OUT/bench.err"; exit 1; }
  echo BENCH_OK
elif [ "$PROF" != "-" ]; then bash profiles/run_profile.sh "$PROF"; fi
