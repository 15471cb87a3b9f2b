#!/bin/bash
# GPU diagnostic: template-kernel times (config 2, 1M Pods) at several minimum
# waves-per-SIMD settings of the JIT (GKGPU_JIT_WPE), alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export GKGPU_JIT_CACHE=/tmp/gkjc
for w in ${@:-2 3 2 3}; do
  GKGPU_JIT_WPE=$w timeout -k 10 200 python -u tools/probe_repeat.py 1000000 > gpurun_out/wpe_$w.log 2>&1 || { echo FAIL $w; tail -20 gpurun_out/wpe_$w.log; exit 1; }
  echo "wpe=$w $(tail -1 gpurun_out/wpe_$w.log)"
done
