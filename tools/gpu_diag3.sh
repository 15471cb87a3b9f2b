#!/bin/bash
# GPU probe: K8sContainerLimits kernel time vs per-lane scratch capacities
# (GK_BCAP byte buffer, GK_HCAP heap words) and waves/SIMD (GKGPU_JIT_WPE).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export GKGPU_JIT_CACHE=0
run() {
  echo "== $1" >> gpurun_out/diag3.log
  timeout -k 10 150 python -u tools/probe_repeat.py 1000000 K8sContainerLimits 2>&1 | tail -3 >> gpurun_out/diag3.log || { echo "FAIL $1"; exit 1; }
}
GKGPU_JIT_PRE= run base
GKGPU_JIT_PRE=GK_BCAP=1024 run bcap1024
GKGPU_JIT_PRE=GK_BCAP=1024,GK_HCAP=64 run bcap1024_hcap64
GKGPU_JIT_WPE=3 GKGPU_JIT_PRE=GK_BCAP=1024,GK_HCAP=64 run wpe3_small
GKGPU_JIT_WPE=4 GKGPU_JIT_PRE=GK_BCAP=512,GK_HCAP=64 run wpe4_small
cat gpurun_out/diag3.log
