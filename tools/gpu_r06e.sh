#!/bin/bash
# Round-6 HEAD record + lane-memory A/B on one MI355X:
#   1. profiles/run_profile.sh (rocprof trace, FETCH/WRITE PMC passes, bench
#      with the CPU baseline) at HEAD, config 2
#   2. per-template lane caps (GK_BCAP / GK_HCAP) and the spill-VGPR
#      preallocation off (GKGPU_JIT_PREALLOC=0) against the defaults, configs 2, 4
#   3. one SQ instruction-mix PMC pass of config 2, run last
#   bash tools/gpu_r06e.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r06e}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export GKGPU_JIT_CACHE=/tmp/gkjit_cache
mkdir -p $GKGPU_JIT_CACHE && cp -n .jitcache/*.co $GKGPU_JIT_CACHE/ 2>/dev/null
bash profiles/run_profile.sh "$TAG" > "$OUT/profile.log" 2>&1 || { echo PROFILE_FAIL; tail "$OUT/profile.log"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('BENCH', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms; e2e', round(d['config']['end_to_end_evals_per_s']/1e6,1), 'M; upload', d['config'].get('upload_bytes'), 'stage', d['config'].get('stage_ms'), 'frac', d['roofline']['frac'], 'traffic', d['roofline']['traffic'])" gpurun_out/prof_$TAG/bench.json
bash tools/gpu_bench_ab.sh ${TAG}_c2 "--steps 20 --warmup 3 --shard-leg off --cpu-e2e off" "" "GKGPU_JIT_PRE=GK_BCAP=1024,GK_HCAP=64" \
  "GKGPU_JIT_PRE=GK_BCAP=512,GK_HCAP=48" "GKGPU_JIT_PREALLOC=0" "" || exit 1
bash tools/gpu_bench_ab.sh ${TAG}_c4 "--config 4 --steps 10 --warmup 2 --cpu-e2e off" "" "GKGPU_JIT_PRE=GK_BCAP=1024,GK_HCAP=64" \
  "GKGPU_JIT_PREALLOC=0" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$GRAFT_REPO_ROOT/$OUT/counters_avail.txt" 2>&1 || echo "counter list rc $?"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES \
  -d "$GRAFT_REPO_ROOT/$OUT/sq1" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --cpu-sample 0 --shard-leg off --cpu-e2e off \
  > "$GRAFT_REPO_ROOT/$OUT/sq1_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/sq1.err"
echo "sq1 rc $?"
