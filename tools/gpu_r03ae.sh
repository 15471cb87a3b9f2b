#!/bin/bash
# Round-3 closing measurement at HEAD: the whole -m gpu suite, then the
# rocprof / PMC / bench sequence for config 2 and for config 6 at 200K objects.
#   bash tools/gpu_r03ae.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03ae}
OUT=gpurun_out/$TAG
mkdir -p "$OUT" gpurun_out/jitcache
cp -n .jitcache/*.co gpurun_out/jitcache/ 2>/dev/null || true
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ]; then echo PYTEST_FAIL $rc; grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20; exit 1; fi
echo PYTEST_OK
bash profiles/run_profile.sh "$TAG" || { echo C2_PROFILE_FAIL; exit 1; }
echo C2_PROFILE_OK
true
true
