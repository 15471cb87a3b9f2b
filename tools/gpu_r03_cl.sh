#!/bin/bash
# K8sContainerLimits cost analysis at 1M Pods (config 2): template variants
# (tools/probe_variants.py), then SQ / cache PMC passes of the full kernel.
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/${1:-r03_cl}
mkdir -p "$OUT" "$ROOT/gpurun_out/jitcache"
cp -n "$ROOT"/.jitcache/*.co "$ROOT/gpurun_out/jitcache/" 2>/dev/null || true
export GKGPU_JIT_CACHE=$ROOT/gpurun_out/jitcache
timeout -k 10 600 python3 -u "$ROOT/tools/probe_variants.py" 1000000 > "$OUT/variants.log" 2>&1 || { echo VARIANTS_FAIL; tail -5 "$OUT/variants.log"; exit 1; }
cat "$OUT/variants.log" | grep backend
cd /tmp && export TMPDIR=/tmp
P=(
 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES"
 "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"
 "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_HIT_sum"
)
i=0
for p in "${P[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $p -d "$OUT/p$i" -o run -- python3 "$ROOT/tools/probe_repeat.py" 1000000 K8sContainerLimits > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i done"
done
