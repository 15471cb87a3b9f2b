#!/bin/bash
# GPU diagnostic: bench with the divergence-aware review order off (0) and on (1), alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export GKGPU_JIT_CACHE=$PWD/.jitcache
b() { GKGPU_SIZE_ORDER=$2 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/ord_$1.json 2>gpurun_out/ord_$1.err && python3 -c "
import json; d=json.load(open('gpurun_out/ord_$1.json')); print('$1', round(d['ms_per_step'],2), [(k['kernel'][-6:], round(k['avg_ms'],2)) for k in d['kernels']])"; }
b off1 0 && b on1 1 && b off2 0 && b on2 1
rocm-smi --showclocks --showtemp --showpower > gpurun_out/smi.txt 2>&1 || true
