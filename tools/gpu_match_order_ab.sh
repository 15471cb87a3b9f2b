#!/bin/bash
# GPU diagnostic: config 2 and config 4 bench with the match-affinity review
# order in mode 1 (signature first) and mode 2 (default: kind, elements, signature, nodes),
# alternated, then the staged-batch parity tests (engine.cc env_mode documents the modes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export GKGPU_JIT_CACHE=$PWD/.jitcache
b() { GKGPU_MATCH_ORDER=$2 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 $3 > gpurun_out/mo_$1.json 2>gpurun_out/mo_$1.err && python3 -c "
import json; d=json.load(open('gpurun_out/mo_$1.json')); print('$1', round(d['value']/1e6,1), round(d['ms_per_step'],2), [(k['kernel'][-6:], round(k['avg_ms'],2)) for k in d['kernels']])"; }
b m1a 1 && b m2a 2 && b m1b 1 && b m2b 2 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "staged or config2_agilebank_pods or config4" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_mo.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_mo.log; [ $rc = 0 ] || exit 1
b c4m1 1 "--config 4" && b c4m2 2 "--config 4"
