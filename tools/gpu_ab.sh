#!/bin/bash
# A/B of the template-kernel switches on config 2 at 1M Pods (tools/probe_repeat.py:
# per-launch kernel ms over 12 sweeps of one staged batch), one process per setting.
#   bash tools/gpu_ab.sh <tag> "<setting>" ["<setting>" ...]   (setting: "" or "VAR=val VAR2=val")
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT" gpurun_out/jitcache
cp -n .jitcache/*.co gpurun_out/jitcache/ 2>/dev/null || true
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jitcache
i=0
for s in "$@"; do
  i=$((i+1))
  echo "== [$i] ${s:-default}" | tee -a "$OUT/ab.log"
  env $s timeout -k 10 300 python3 -u tools/probe_repeat.py 1000000 >> "$OUT/ab.log" 2>&1 || { echo "AB_FAIL [$i]"; tail -5 "$OUT/ab.log"; exit 1; }
  grep "step 11" "$OUT/ab.log" | tail -1
done
