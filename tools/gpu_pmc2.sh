#!/bin/bash
# PMC passes (instruction fetch / cache) over the K8sContainerLimits kernel.
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/pmc2
mkdir -p "$OUT"
export GKGPU_JIT_CACHE=$ROOT/.jitcache
cd /tmp && export TMPDIR=/tmp
P=(
 "SQ_IFETCH SQ_IFETCH_LEVEL SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY"
 "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_REQ SQC_ICACHE_MISSES_DUPLICATE"
)
i=0
for p in "${P[@]}"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $p -d "$OUT/p$i" -o run -- python3 "$ROOT/tools/probe_repeat.py" 1000000 K8sContainerLimits > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i done"
done
