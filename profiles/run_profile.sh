#!/bin/bash
# Profiles the audit-sweep bench on an MI355X (run from the repo root on the GPU box):
#   bash profiles/run_profile.sh r01
# 1. rocprofv3 --kernel-trace --stats of a short bench run (per-kernel durations)
# 2. two PMC passes, FETCH_SIZE then WRITE_SIZE (they do not share a TCC pass)
# 3. HBM bytes per launch from those passes (summarize.py --traffic-only)
# 4. bench.py (default config, CPU baseline included), reading the traffic of 3
# Outputs land in gpurun_out/prof_<round>/; the summaries worth keeping are
# copied into profiles/ afterwards (python profiles/summarize.py gpurun_out/prof_<round> <round>).
set -eo pipefail
R=${1:-r01}
ROOT=$PWD
OUT=$ROOT/gpurun_out/prof_$R
mkdir -p "$OUT"
export GKGPU_JIT_CACHE=$ROOT/.jitcache
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 1 --cpu-sample 0 > "$OUT/bench_trace.json"
echo "trace done"
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run -- \
  python3 "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-sample 0 > "$OUT/bench_fetch.json"
echo "fetch done"
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run -- \
  python3 "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-sample 0 > "$OUT/bench_write.json"
echo "write done"
python3 "$ROOT/profiles/summarize.py" --traffic-only "$OUT"
timeout -k 10 500 python3 "$ROOT/bench.py" --traffic-json "$OUT/traffic.json" > "$OUT/bench.json"
echo "bench done"
