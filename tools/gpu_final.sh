#!/bin/bash
# Round-end record on one MI355X: part "a" = the GPU suite and the config-2
# profile (rocprof trace + PMC passes + bench with the CPU baseline); part "b" =
# the other configurations' bench lines (CPU baselines included), config 5
# coalesced, and the from-cache sweep at 1M synced Pods.
#   bash tools/gpu_final.sh <tag> a|b
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; PART=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
# template-kernel code objects: a cache outside gpurun_out/ seeded with the
# tree's .jitcache (A/B variants compile many kernels; gpurun pulls back at
# most 64 MiB), the new ones copied back to gpurun_out/jitcache_new at exit
JC=${GKGPU_JIT_CACHE:-/tmp/gkjit_cache}
mkdir -p "$JC"
cp -n .jitcache/*.co "$JC/" 2>/dev/null || true
export GKGPU_JIT_CACHE=$JC
jit_pull() {
  local new=() f sz=0
  for f in "$JC"/*.co; do [ -e ".jitcache/$(basename "$f")" ] || { new+=("$f"); sz=$((sz + $(stat -c %s "$f"))); }; done
  if [ ${#new[@]} -gt 0 ] && [ $sz -lt 40000000 ]; then mkdir -p gpurun_out/jitcache_new && cp -n "${new[@]}" gpurun_out/jitcache_new/; fi
  echo "jit cache: ${#new[@]} new code objects, $sz bytes"
}
trap jit_pull EXIT
if [ "$PART" = a ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc = 0 ] || exit 1
  bash profiles/run_profile.sh "$TAG" > "$OUT/profile.log" 2>&1 || { echo PROFILE_FAIL; tail "$OUT/profile.log"; exit 1; }
  echo profile done
else
  for c in 3 4 6; do
    timeout -k 10 400 python -u bench.py --config $c > "$OUT/c$c.json" 2> "$OUT/c$c.err" || { echo "C${c}_FAIL"; tail "$OUT/c$c.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('C$c', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms; cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value']/1e6,1))" "$OUT/c$c.json"
  done
  timeout -k 10 300 python -u bench.py --config 5 > "$OUT/c5.json" 2> "$OUT/c5.err" || { echo C5_FAIL; tail "$OUT/c5.err"; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('C5', d['config']['latency_ms'], round(d['value']/1e6,2), 'M/s; cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value']/1e6,2))" "$OUT/c5.json"
  timeout -k 10 300 python -u bench.py --config 5 --coalesce-us 300 --rate 20000 --steps 400 > "$OUT/c5_coal.json" 2> "$OUT/c5_coal.err" || { echo C5C_FAIL; tail "$OUT/c5_coal.err"; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('C5COAL', round(c['requests_per_s']), 'req/s', c['latency_ms'], c['mean_requests_per_launch'])" "$OUT/c5_coal.json"
  timeout -k 10 600 python -u bench.py --from-cache --steps 3 --warmup 1 > "$OUT/cache.json" 2> "$OUT/cache.err" || { echo CACHE_FAIL; tail "$OUT/cache.err"; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('CACHE', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],1), 'ms', c['results_per_audit'], c['first_audit_s'], c['steady_timing_ms'])" "$OUT/cache.json"
fi
