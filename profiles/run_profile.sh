#!/bin/bash
# Profiles the audit-sweep bench on an MI355X (run from the repo root on the GPU box):
#   bash profiles/run_profile.sh r01
# 1. bench.py (default config, CPU baseline included)
# 2. rocprofv3 --kernel-trace --stats of a short bench run (per-kernel durations)
# 3. two PMC passes, FETCH_SIZE then WRITE_SIZE (they do not share a TCC pass)
# Outputs land in gpurun_out/prof_<round>/; the summaries worth keeping are
# copied into profiles/ afterwards.
set -eo pipefail
R=${1:-r01}
ROOT=$PWD
OUT=$ROOT/gpurun_out/prof_$R
mkdir -p "$OUT"
export GKGPU_JIT_CACHE=$ROOT/.jitcache
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 python3 "$ROOT/bench.py" > "$OUT/bench.json"
echo "bench done"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 1 --cpu-sample 0 > "$OUT/bench_trace.json"
echo "trace done"
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run -- \
  python3 "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-sample 0 > "$OUT/bench_fetch.json"
echo "fetch done"
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run -- \
  python3 "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-sample 0 > "$OUT/bench_write.json"
echo "write done"
