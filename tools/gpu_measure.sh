#!/bin/bash
# One GPU call of measurements after the suite: same-call A/Bs of JIT
# switches on config 2 (and config 4), the config-5 phase breakdown and batch
# bench, and the from-cache bench.  Summaries print as AB lines; JSON under
# gpurun_out/<tag>/.   bash tools/gpu_measure.sh <tag> [c2|c4|c5|cache ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04m}; shift
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
for what in "${@:-c2 c4 c5 cache}"; do
  case $what in
    c2) bash tools/gpu_bench_ab.sh "$TAG/c2" "--steps 10 --warmup 2" "" "GKGPU_CONCURRENT=0" \
          "GKGPU_JIT_WPE=2 GKGPU_LDS_HEAP=16" "GKGPU_JIT_WPE=2 GKGPU_LDS_HEAP=16 GKGPU_CONCURRENT=0" || exit 1 ;;
    c5t) GKGPU_FLATTEN_TRACE=2 timeout -k 10 120 python -u tools/probe_c5_time.py 256 > "$OUT/c5t.txt" 2>&1 || { echo C5T_FAIL; tail "$OUT/c5t.txt"; exit 1; }
        grep -E "flatten_reviews|intern|relocate" "$OUT/c5t.txt" | tail -8; tail -3 "$OUT/c5t.txt" ;;
    sets) bash tools/gpu_bench_ab.sh "$TAG/sets" "--steps 10 --warmup 2" "" "GKGPU_REGO_SETS=0" || exit 1
          bash tools/gpu_bench_ab.sh "$TAG/sets4" "--config 4 --steps 5 --warmup 1" "" "GKGPU_REGO_SETS=0" || exit 1 ;;
    bch) bash tools/gpu_bench_ab.sh "$TAG/bch" "--steps 10 --warmup 2" "" "GKGPU_JIT_PRE=GK_BCHUNK=0" "GKGPU_REGO_SETS=3" || exit 1
         bash tools/gpu_bench_ab.sh "$TAG/bch4" "--config 4 --steps 5 --warmup 1" "" "GKGPU_JIT_PRE=GK_BCHUNK=0" "GKGPU_REGO_SETS=3" || exit 1 ;;
    c5pmc) R=$PWD; ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INSTS_LDS \
             -d "$R/$OUT/c5pmc" -o run -- python3 "$R/tools/probe_c5_time.py" 256 ) > "$OUT/c5pmc.log" 2>&1 || { echo C5PMC_FAIL; tail "$OUT/c5pmc.log"; exit 1; }
           python3 tools/pmc_table.py "$OUT/c5pmc" | tee "$OUT/c5pmc.txt"; rm -rf "$OUT/c5pmc" ;;
    rememo) bash tools/gpu_bench_ab.sh "$TAG/rememo4" "--config 4 --steps 5 --warmup 1" "" "GKGPU_RE_MEMO=0" || exit 1
            bash tools/gpu_bench_ab.sh "$TAG/rememo3" "--config 3 --steps 5 --warmup 1" "" "GKGPU_RE_MEMO=0" || exit 1 ;;
    c5c) for r in 20000 40000; do
           timeout -k 10 300 python -u bench.py --config 5 --coalesce-us 300 --rate $r --steps 400 --cpu-sample 0 > "$OUT/c5c_$r.json" 2> "$OUT/c5c_$r.err" || { echo C5C_FAIL; tail "$OUT/c5c_$r.err"; exit 1; }
           python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('C5COAL', sys.argv[2], round(c['requests_per_s']), 'req/s', {k: round(v, 3) for k, v in c['latency_ms'].items()}, round(c['mean_requests_per_launch'], 1))" "$OUT/c5c_$r.json" $r
         done ;;
    fmt) bash tools/gpu_bench_ab.sh "$TAG/fmt" "--steps 10 --warmup 2" "" "GKGPU_FMT_WIDE=0" || exit 1
         for v in 1 0; do
           GKGPU_FMT_WIDE=$v timeout -k 10 300 python -u bench.py --config 5 --steps 1000 --warmup 20 --cpu-sample 0 > "$OUT/c5w$v.json" 2> "$OUT/c5w$v.err" || { echo C5W_FAIL; tail "$OUT/c5w$v.err"; exit 1; }
           python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('C5W', sys.argv[2], {k: round(v, 3) for k, v in c['latency_ms'].items()}, round(d['value']/1e6,2), 'M/s', [round(x, 3) for x in c['kernel_ms_last_launch']])" "$OUT/c5w$v.json" $v
         done ;;
    heap) bash tools/gpu_bench_ab.sh "$TAG/heap" "--steps 10 --warmup 2" "" "GKGPU_LDS_HEAP=32" || exit 1
          bash tools/gpu_bench_ab.sh "$TAG/heap4" "--config 4 --steps 5 --warmup 1" "" "GKGPU_LDS_HEAP=32" || exit 1 ;;
    fst) bash tools/gpu_bench_ab.sh "$TAG/fst" "--steps 10 --warmup 2" "" "GKGPU_FMT_STAGE=16384" || exit 1
         bash tools/gpu_bench_ab.sh "$TAG/fst4" "--config 4 --steps 5 --warmup 1" "" "GKGPU_FMT_STAGE=16384" || exit 1 ;;
    c24) bash tools/gpu_bench_ab.sh "$TAG/c24" "--steps 10 --warmup 2" "" || exit 1
         bash tools/gpu_bench_ab.sh "$TAG/c24_4" "--config 4 --steps 5 --warmup 1" "" || exit 1 ;;
    suite) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
          tail -4 "$OUT/pytest_gpu.log"; [ $rc = 0 ] || exit 1 ;;
    c2t) GKGPU_FLATTEN_TRACE=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 > "$OUT/c2t.json" 2> "$OUT/c2t.err" || { echo C2T_FAIL; tail "$OUT/c2t.err"; exit 1; }
        grep -E "flatten|stage upload|intern" "$OUT/c2t.err" | tail -12
        python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('C2T', round(d['value']/1e6,1), 'M/s stage_s', c['stage_s'], c['stage_ms'], 'prepare_s', c.get('prepare_s'), 'e2e', round(c['end_to_end_evals_per_s']/1e6,2))" "$OUT/c2t.json" ;;
    p4) ( bash profiles/run_profile.sh "${TAG}_c4" --config 4 ) > "$OUT/p4.log" 2>&1 || { echo P4_FAIL; tail "$OUT/p4.log"; exit 1; }
        tail -5 "$OUT/p4.log" ;;
    p2) ( bash profiles/run_profile.sh "${TAG}" ) > "$OUT/p2.log" 2>&1 || { echo P2_FAIL; tail "$OUT/p2.log"; exit 1; }
        tail -3 "$OUT/p2.log" ;;
    c4) bash tools/gpu_bench_ab.sh "$TAG/c4" "--config 4 --steps 5 --warmup 1" "" "GKGPU_CONCURRENT=0" \
          "GKGPU_JIT_WPE=2 GKGPU_LDS_HEAP=16 GKGPU_CONCURRENT=0" || exit 1 ;;
    c5) timeout -k 10 300 python -u tools/probe_c5_time.py 256 > "$OUT/c5_phases.txt" 2>&1 || { echo C5P_FAIL; tail "$OUT/c5_phases.txt"; exit 1; }
        cat "$OUT/c5_phases.txt"
        timeout -k 10 300 python -u bench.py --config 5 --steps 1000 --warmup 20 > "$OUT/c5_batch.json" 2> "$OUT/c5_batch.err" || { echo C5_FAIL; tail "$OUT/c5_batch.err"; exit 1; }
        python -c "import json,sys; d=json.load(open(sys.argv[1])); print('C5', d['config']['latency_ms'], round(d['value']/1e6,2), 'M/s; cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value']/1e6,2))" "$OUT/c5_batch.json" ;;
    cache) timeout -k 10 600 python -u bench.py --from-cache --steps 3 --warmup 1 > "$OUT/cache.json" 2> "$OUT/cache.err" || { echo CACHE_FAIL; tail "$OUT/cache.err"; exit 1; }
        python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('CACHE', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],1), 'ms', c['results_per_audit'], c['cache_builds'], c['first_audit_s'], c['steady_timing_ms'])" "$OUT/cache.json" ;;
  esac
done
