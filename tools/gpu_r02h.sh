#!/bin/bash
# A/B in one call: (1) JIT memo registers (GKGPU_JIT_MEMO2 / GKGPU_JIT_LMEMO) on
# K8sContainerLimits and config 2; (2) review order modes on config 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02h
export GKGPU_JIT_CACHE=$PWD/.jitcache
run() { local tag=$1; shift; env "$@" timeout -k 10 240 python -u tools/probe_repeat.py 1000000 $ONLY > gpurun_out/r02h/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/r02h/$tag.log; exit 1; }; echo "$tag: $(tail -1 gpurun_out/r02h/$tag.log)"; }
ONLY=K8sContainerLimits
run cl_base X=1
run cl_nom2 GKGPU_JIT_MEMO2=0
run cl_nolm GKGPU_JIT_LMEMO=0
run cl_base2 X=1
ONLY=""
run all_base X=1
run all_nom2 GKGPU_JIT_MEMO2=0
run all_nolm GKGPU_JIT_LMEMO=0
for m in 0 1 2; do
  GKGPU_MATCH_ORDER=$m timeout -k 10 300 python -u bench.py --config 4 --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/r02h/c4_m$m.json 2> gpurun_out/r02h/c4_m$m.err || { tail -5 gpurun_out/r02h/c4_m$m.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r02h/c4_m$m.json').read().strip().splitlines()[-1])
print('c4 mode $m', round(d['value']/1e6,1), 'M evals/s', [(k['kernel'][:12], round(k['avg_ms'],2)) for k in d['kernels']])"
done
