#!/bin/bash
# Host-trap PC sampling of one template kernel (default K8sContainerLimits) at
# 1M Pods: where the waves of the predicate spend their time.
#   bash tools/gpu_pcsample.sh <tag> [kind]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03pc}
KIND=${2:-K8sContainerLimits}
ROOT=$PWD
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT" gpurun_out/jitcache
cp -n .jitcache/*.co gpurun_out/jitcache/ 2>/dev/null || true
export GKGPU_JIT_CACHE=$ROOT/gpurun_out/jitcache
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval 50 --output-format csv -d "$OUT/pc" -o run -- \
  python3 "$ROOT/tools/probe_repeat.py" 1000000 "$KIND" > "$OUT/pc.log" 2>&1 || { echo PC_FAIL; tail -20 "$OUT/pc.log"; exit 1; }
echo PC_OK
find "$OUT/pc" -name "*.csv" | head
