#!/bin/bash
# Round-6 HEAD record: GPU suite, config-2 profile (rocprof trace + PMC + bench
# with the CPU baseline), then the column form's staging trace.
#   bash tools/gpu_r06h.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r06h}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export GKGPU_JIT_CACHE=/tmp/gkjit_cache
mkdir -p $GKGPU_JIT_CACHE && cp -n .jitcache/*.co $GKGPU_JIT_CACHE/ 2>/dev/null
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc = 0 ] || exit 1
bash profiles/run_profile.sh "$TAG" > "$OUT/profile.log" 2>&1 || { echo PROFILE_FAIL; tail "$OUT/profile.log"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('BENCH', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms; e2e', round(c['end_to_end_evals_per_s']/1e6,1), 'M; upload', c.get('upload_bytes'), 'stage', c.get('stage_ms'), 'frac', d['roofline']['frac'], 'traffic', d['roofline']['traffic'], 'c4', round((d.get('config4_shard') or {}).get('value', 0)/1e6, 1))" gpurun_out/prof_$TAG/bench.json
GKGPU_FLATTEN_TRACE=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 --shard-leg off --cpu-e2e off > "$OUT/trace.json" 2> "$OUT/trace.err" || { echo TRACE_FAIL; tail "$OUT/trace.err"; exit 1; }
grep -E "^columns|^upload|^stage|^flatten: (parse|intern|device)" "$OUT/trace.err" | tail -14
