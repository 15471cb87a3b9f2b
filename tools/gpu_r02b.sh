#!/bin/bash
# Round-2 perf probe on K8sContainerLimits (config 2, 1M Pods): per-step kernel
# time A/B of per-template lane capacities and the unrolled member scan
# (GKGPU_JIT_PRE defines), then PMC passes on the default build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02b
export GKGPU_JIT_CACHE=$PWD/.jitcache
rocm-smi --showclocks > gpurun_out/r02b/clocks_before.txt 2>&1 || true
run() { GKGPU_JIT_PRE="$2" timeout -k 10 240 python -u tools/probe_repeat.py 1000000 K8sContainerLimits > gpurun_out/r02b/$1.log 2>&1 || { echo "FAIL $1"; tail -5 gpurun_out/r02b/$1.log; exit 1; }; echo "$1: $(tail -1 gpurun_out/r02b/$1.log)"; }
run A ""
run B "GK_BCAP=512,GK_HCAP=16,GK_EMCAP=16"
run C "GK_BCAP=512,GK_HCAP=16,GK_EMCAP=16,GK_VGET_UNROLL=1"
run D "GK_VGET_UNROLL=1"
run A2 ""
rocm-smi --showclocks > gpurun_out/r02b/clocks_after.txt 2>&1 || true
cd /tmp && export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
P=(
 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES"
 "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"
 "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"
 "FETCH_SIZE"
 "WRITE_SIZE"
)
i=0
for p in "${P[@]}"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $p -d "$ROOT/gpurun_out/r02b/p$i" -o run -- python3 "$ROOT/tools/probe_repeat.py" 1000000 K8sContainerLimits > "$ROOT/gpurun_out/r02b/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$ROOT/gpurun_out/r02b/p$i.log"; exit 1; }
  echo "pass $i done"
done
