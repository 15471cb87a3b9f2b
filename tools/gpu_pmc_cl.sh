#!/bin/bash
# PMC passes over the K8sContainerLimits kernel (config 2, 1M Pods): where the
# wave cycles go (issue vs wait), instruction mix and cache behaviour.
set -eo pipefail
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/pmc_cl
mkdir -p "$OUT"
export GKGPU_JIT_CACHE=$ROOT/.jitcache
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
echo listed
P=(
 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES"
 "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"
 "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_HIT_sum TCC_MISS_sum"
)
i=0
for p in "${P[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $p -d "$OUT/p$i" -o run -- python3 "$ROOT/tools/probe_repeat.py" 1000000 K8sContainerLimits > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; }
  echo "pass $i done"
done
