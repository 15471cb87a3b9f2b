#!/bin/bash
# config-4 flagged reviews at HEAD: new memo hash vs the round-2 mixers vs memo off
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03t
mkdir -p "$OUT" gpurun_out/jitcache
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jitcache
for v in "" GKGPU_JIT_PRE=GK_GM_HASH_OLD=1 GKGPU_GMEMO=0 GKGPU_MEMO_NODES=0; do
  echo "== $v"
  env $v timeout -k 10 240 python -u tools/probe_flags.py 4 1250000 > "$OUT/flags_$(echo ${v:-default} | tr '=' '_').log" 2>&1 || { echo PROBE_FAIL; exit 1; }
  grep -E "sweep|flagged|reasons|kinds|example" "$OUT/flags_$(echo ${v:-default} | tr '=' '_').log" | cut -c1-600
done
