#!/bin/bash
# Round-5 GPU calls: bash tools/gpu_r05.sh <tag> <step> [<step> ...]
#   suite  the GPU test suite
#   bench  the default bench line (config 2 + config4_shard + CPU end to end)
#   early  GKGPU_FN_EARLY A/B on configs 2 and 4
#   ab2 "<settings>..." / ab4: same-call A/Bs (settings in AB2 / AB4 env, ';'-separated)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
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
for what in "$@"; do
  case $what in
    suite) timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
           tail -4 "$OUT/pytest_gpu.log"; [ $rc = 0 ] || exit 1 ;;
    bench) timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo BENCH_FAIL; tail "$OUT/bench.err"; exit 1; }
           python - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c = d["config"]
print("BENCH", round(d["value"] / 1e6, 1), "M/s", round(d["ms_per_step"], 3), "ms; frac", d["roofline"]["frac"],
      "e2e", round(c["end_to_end_evals_per_s"] / 1e6, 2), "stage", c["stage_s"])
cb = d["cpu_baseline"] or {}
print("CPU", cb.get("value"), "e2e", (cb.get("end_to_end") or {}).get("value"))
s = d.get("config4_shard") or {}
print("SHARD4", s.get("value"), s.get("ms_per_step"), s.get("fallback_reviews"), (s.get("roofline") or {}).get("frac"), s.get("kernels"))
PY
           ;;
    parity) timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_audit_cache.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_parity.log" 2>&1; rc=$?
           tail -4 "$OUT/pytest_parity.log"; [ $rc = 0 ] || exit 1 ;;
    audit) timeout -k 10 900 python -u -m pytest tests/test_audit_cache.py tests/test_audit_writer.py tests/test_parallel_gpu.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_audit.log" 2>&1; rc=$?
           tail -4 "$OUT/pytest_audit.log"; [ $rc = 0 ] || exit 1 ;;
    scale) timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 400 --timeout-method thread > "$OUT/pytest_scale.log" 2>&1; rc=$?
           tail -4 "$OUT/pytest_scale.log"; [ $rc = 0 ] || exit 1 ;;
    scale4) timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q -k config4 --timeout 300 --timeout-method thread > "$OUT/pytest_scale4.log" 2>&1; rc=$?
           tail -4 "$OUT/pytest_scale4.log"; grep -E "^E " "$OUT/pytest_scale4.log" | head -5; [ $rc = 0 ] || exit 1 ;;
    early) bash tools/gpu_bench_ab.sh "$TAG/early2" "--steps 10 --warmup 2 --shard-leg off" "" "GKGPU_FN_EARLY=1" || exit 1
           bash tools/gpu_bench_ab.sh "$TAG/early4" "--config 4 --steps 5 --warmup 1" "" "GKGPU_FN_EARLY=1" || exit 1 ;;
    ab2) IFS=';' read -ra S <<< "$AB2"; bash tools/gpu_bench_ab.sh "$TAG/ab2" "--steps 10 --warmup 2 --shard-leg off" "${S[@]}" || exit 1 ;;
    ab4) IFS=';' read -ra S <<< "$AB4"; bash tools/gpu_bench_ab.sh "$TAG/ab4" "--config 4 --steps 5 --warmup 1" "${S[@]}" || exit 1 ;;
    ab6) IFS=';' read -ra S <<< "$AB6"; bash tools/gpu_bench_ab.sh "$TAG/ab6" "--config 6 --steps 5 --warmup 1 --shard-leg off" "${S[@]}" || exit 1 ;;
    ab3) IFS=';' read -ra S <<< "$AB3"; bash tools/gpu_bench_ab.sh "$TAG/ab3" "--config 3 --steps 5 --warmup 1 --shard-leg off" "${S[@]}" || exit 1 ;;
    quick) timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --shard-leg off --cpu-sample 0 > "$OUT/quick.json" 2> "$OUT/quick.err" || { echo QUICK_FAIL; tail "$OUT/quick.err"; exit 1; }
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config']; print('QUICK', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms kernels', round(c['kernel_ms_per_step'],3))" "$OUT/quick.json" ;;
    cache) timeout -k 10 600 python -u bench.py --from-cache --steps 5 --warmup 1 > "$OUT/cache.json" 2> "$OUT/cache.err" || { echo CACHE_FAIL; tail "$OUT/cache.err"; exit 1; }
        python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('CACHE', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms', c['results_per_audit'], c['first_audit_s'], c['steady_timing_ms'], 'decode-all', c['decode_all_rows_ms'])" "$OUT/cache.json" ;;
    sq) # SQ / TCP / TA counters of a short config-2 bench, one rocprofv3 pass per set
        R=$PWD; i=0
        for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
                   "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" \
                   "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_FLAT_READ_WAVEFRONTS_sum TA_FLAT_WRITE_WAVEFRONTS_sum" \
                   ${SQ_EXTRA:+"$SQ_EXTRA"}; do
          i=$((i+1))
          ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pmc $set -d "$R/$OUT/sq$i" -o run -- \
              python3 "$R/bench.py" --steps 2 --warmup 1 --cpu-sample 0 --shard-leg off $SQ_ARGS ) > "$OUT/sq$i.log" 2>&1; rc=$?
          if [ $rc != 0 ]; then echo "SQ pass $i rc $rc"; tail -3 "$OUT/sq$i.log"; case $rc in 124|134|137|139) exit 1;; esac; continue; fi
          python3 tools/pmc_table.py "$OUT/sq$i" | tee "$OUT/sq$i.txt"; rm -rf "$OUT/sq$i"
        done ;;
    p2) ( bash profiles/run_profile.sh "${TAG}" ) > "$OUT/p2.log" 2>&1 || { echo P2_FAIL; tail "$OUT/p2.log"; exit 1; }
        tail -3 "$OUT/p2.log" ;;
  esac
done
