#!/bin/bash
# re_match cross-lane memo: regex parity tests, then config 3 with and without it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02ae
export GKGPU_JIT_CACHE=$PWD/.jitcache
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread -k "regex or config3 or integration or kat" > gpurun_out/r02ae/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r02ae/pytest.log
[ $rc -eq 0 ] || exit $rc
for m in 0 1; do
  GKGPU_RE_MEMO=$m timeout -k 10 400 python -u bench.py --config 3 --cpu-sample 0 --steps 5 > gpurun_out/r02ae/c3_m$m.json 2> gpurun_out/r02ae/c3_m$m.err || exit 1
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/r02ae/c3_m$m.json').read().strip().splitlines()[-1])
print('memo $m', round(d['value']/1e6,1), 'M evals/s', round(d['ms_per_step'],2), 'ms', [(k['kernel'][:10], round(k['avg_ms'],2)) for k in d['kernels']])"
done
exit $rc
