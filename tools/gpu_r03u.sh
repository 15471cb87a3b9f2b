#!/bin/bash
# config-4 flagged reviews (new vs round-2 memo hash), then config 5 batch and
# config 2 kernel times with the scratch-free size/format passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03u
mkdir -p "$OUT" gpurun_out/jitcache
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jitcache
for v in "" GKGPU_JIT_PRE=GK_GM_HASH_OLD=1; do
  f="$OUT/flags_$(echo ${v:-default} | tr '=' '_').log"
  echo "== $v"
  env $v timeout -k 10 240 python -u tools/probe_flags.py 4 1250000 > "$f" 2>&1 || { echo PROBE_FAIL; tail -3 "$f"; exit 1; }
  grep -E "sweep|flagged|reasons|kinds|example" "$f" | cut -c1-700
done
timeout -k 10 300 python -u bench.py --config 5 --steps 500 --warmup 20 --cpu-sample 0 > "$OUT/c5_batch.json" 2> "$OUT/c5_batch.err" || { echo C5_FAIL; tail "$OUT/c5_batch.err"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c5_batch.json')); c=d['config']; print('c5', c['latency_ms'], c['kernel_ms_last_launch'])"
timeout -k 10 300 python3 -u tools/probe_repeat.py 1000000 > "$OUT/repeat.log" 2>&1 || { echo REPEAT_FAIL; tail -3 "$OUT/repeat.log"; exit 1; }
grep "step 11" "$OUT/repeat.log"
timeout -k 10 400 python -u bench.py --config 6 --steps 5 --warmup 1 > "$OUT/c6.json" 2> "$OUT/c6.err" || { echo C6_FAIL; tail "$OUT/c6.err"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c6.json')); c=d['config']; print('c6', d['value'], d['ms_per_step'], c['fallback_reviews'], c['error_reviews'], [(k['kernel'], round(k['avg_ms'],3)) for k in d['kernels']])"
