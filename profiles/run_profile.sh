#!/bin/bash
# Profiles the audit-sweep bench on an MI355X (run from the repo root on the GPU box):
#   bash profiles/run_profile.sh r01 [extra bench.py arguments, e.g. --config 4]
# 1. rocprofv3 --kernel-trace --stats of a short bench run (per-kernel durations)
# 2. two PMC passes, FETCH_SIZE then WRITE_SIZE (they do not share a TCC pass)
# 3. HBM bytes per launch from those passes (summarize.py --traffic-only)
# 4. bench.py (default config, CPU baseline included), reading the traffic of 3
# Outputs land in gpurun_out/prof_<round>/; the summaries worth keeping are
# copied into profiles/ afterwards (python profiles/summarize.py gpurun_out/prof_<round> <round>).
set -eo pipefail
R=${1:-r01}
shift || true
XA=("$@")
ROOT=$PWD
OUT=$ROOT/gpurun_out/prof_$R
mkdir -p "$OUT"
# template-kernel code objects: the tree's .jitcache plus new ones under gpurun_out/
if [ -z "$GKGPU_JIT_CACHE" ]; then mkdir -p /tmp/gkjit_cache; cp -n "$ROOT"/.jitcache/*.co /tmp/gkjit_cache/ 2>/dev/null || true; export GKGPU_JIT_CACHE=/tmp/gkjit_cache; fi
cd /tmp && export TMPDIR=/tmp
# GPU clocks around the run (box-to-box variance: compare only inside one call)
rocm-smi --showclocks > "$OUT/clocks_before.txt" 2>&1 || true
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 1 --cpu-sample 0 --shard-leg off "${XA[@]}" > "$OUT/bench_trace.json"
echo "trace done"
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run -- \
  python3 "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-sample 0 --shard-leg off "${XA[@]}" > "$OUT/bench_fetch.json"
echo "fetch done"
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run -- \
  python3 "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-sample 0 --shard-leg off "${XA[@]}" > "$OUT/bench_write.json"
echo "write done"
python3 "$ROOT/profiles/summarize.py" --traffic-only "$OUT"
# sample the clocks while the bench runs (killed by its PID afterwards)
( while :; do date +%T; rocm-smi --showclocks 2>&1 | grep -E "sclk|mclk|fclk"; sleep 2; done ) > "$OUT/clocks_during.txt" &
SAMPLER=$!
timeout -k 10 500 python3 "$ROOT/bench.py" --traffic-json "$OUT/traffic.json" "${XA[@]}" > "$OUT/bench.json"
kill $SAMPLER 2>/dev/null || true
echo "bench done"
rocm-smi --showclocks > "$OUT/clocks_after.txt" 2>&1 || true
