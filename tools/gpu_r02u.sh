#!/bin/bash
# Inventory-join + guard parity (EMCAP 64), staging trace of the bench, SQ
# instruction counters of K8sContainerLimits, and a vget-unroll A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02u
export GKGPU_JIT_CACHE=$PWD/.jitcache
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread -k "unique_service or guard_program" > gpurun_out/r02u/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r02u/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
GKGPU_FLATTEN_TRACE=1 timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 5 > gpurun_out/r02u/bench.json 2> gpurun_out/r02u/bench.err || exit 1
grep -h "flatten:\|intern_parts\|upload" gpurun_out/r02u/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_LDS SQ_WAVE_CYCLES -d $GRAFT_REPO_ROOT/gpurun_out/r02u/pmc -o run -- python3 $GRAFT_REPO_ROOT/tools/probe_repeat.py 1000000 K8sContainerLimits > $GRAFT_REPO_ROOT/gpurun_out/r02u/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/r02u/pmc.log; }
cd "$GRAFT_REPO_ROOT"
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u tools/probe_repeat.py 1000000 K8sContainerLimits > gpurun_out/r02u/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/r02u/$tag.log; exit 1; }; echo "$tag: $(tail -2 gpurun_out/r02u/$tag.log | head -1)"; }
run cl_base X=1
run cl_unroll GKGPU_JIT_PRE=GK_VGET_UNROLL=1
exit $rc
