#!/bin/bash
# Round-6 final HEAD record: config-2 profile (rocprof trace + PMC + bench with
# the CPU baseline and the config-4 shard leg), SQ instruction mix, staging trace.
#   bash tools/gpu_r06l.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r06l}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export GKGPU_JIT_CACHE=/tmp/gkjit_cache
mkdir -p $GKGPU_JIT_CACHE && cp -n .jitcache/*.co $GKGPU_JIT_CACHE/ 2>/dev/null
bash profiles/run_profile.sh "$TAG" > "$OUT/profile.log" 2>&1 || { echo PROFILE_FAIL; tail "$OUT/profile.log"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('BENCH', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms; e2e', round(c['end_to_end_evals_per_s']/1e6,1), 'M; stage', c.get('stage_ms'), 'frac', d['roofline']['frac'], 'traffic', d['roofline']['traffic'], 'c4', round((d.get('config4_shard') or {}).get('value', 0)/1e6, 1), 'cpu', (d.get('cpu_baseline') or {}).get('value'))" gpurun_out/prof_$TAG/bench.json
GKGPU_FLATTEN_TRACE=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 --shard-leg off --cpu-e2e off > "$OUT/trace.json" 2> "$OUT/trace.err" || { echo TRACE_FAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES \
  -d "$GRAFT_REPO_ROOT/$OUT/sq1" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --cpu-sample 0 --shard-leg off --cpu-e2e off \
  > "$GRAFT_REPO_ROOT/$OUT/sq1_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/sq1.err"
echo "sq1 rc $?"
