#!/bin/bash
# Round-3 GPU check of selected test files (verbose, unbuffered), then the
# profile sequence (rocprof trace + PMC passes + bench) of profiles/run_profile.sh.
#   bash tools/gpu_r03_files.sh <tag> <profile-tag|-> <test files...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; PROF=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT" gpurun_out/jitcache
cp -n .jitcache/*.co gpurun_out/jitcache/ 2>/dev/null || true
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v -s --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -5 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ]; then echo PYTEST_FAIL $rc; grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20; exit 1; fi
echo PYTEST_OK
if [ "$PROF" != "-" ]; then bash profiles/run_profile.sh "$PROF"; fi
