#!/bin/bash
# GPU suite at HEAD (set/emit fast paths, radix review order, parallel intern,
# pinned bounce upload), then the bench with and without the pinned upload.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02p
export GKGPU_JIT_CACHE=$PWD/.jitcache
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r02p/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r02p/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
GKGPU_FLATTEN_TRACE=1 timeout -k 10 300 python -u bench.py --cpu-sample 0 > gpurun_out/r02p/bench_pin1.json 2> gpurun_out/r02p/bench_pin1.err || exit 1
GKGPU_FLATTEN_TRACE=1 GKGPU_PINNED_UPLOAD=0 timeout -k 10 300 python -u bench.py --cpu-sample 0 > gpurun_out/r02p/bench_pin0.json 2> gpurun_out/r02p/bench_pin0.err || exit 1
grep -h "flatten:\|intern_parts" gpurun_out/r02p/bench_pin1.err
python3 -c "
import json
for t in ('pin1','pin0'):
    d=json.load(open('gpurun_out/r02p/bench_%s.json'%t)); c=d['config']
    print(t, round(d['value']/1e6,1), 'M evals/s', c['stage_s'], c['stage_ms'], 'e2e', round(c['end_to_end_evals_per_s']/1e6,2), [ (k['kernel'][:8], round(k['avg_ms'],2)) for k in d['kernels']])
"
exit $rc
