#!/bin/bash
# Occupancy A/B on config 2 (1M Pods): LDS heap words x waves per SIMD the
# template kernels are compiled for (LDS caps blocks per CU; VGPRs cap waves).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02s
export GKGPU_JIT_CACHE=$PWD/.jitcache
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u tools/probe_repeat.py 1000000 > gpurun_out/r02s/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/r02s/$tag.log; exit 1; }; echo "$tag: $(tail -2 gpurun_out/r02s/$tag.log | head -1)"; }
run h32w2 X=1
run h16w2 GKGPU_LDS_HEAP=16
run h16w3 GKGPU_LDS_HEAP=16 GKGPU_JIT_WPE=3
run h16w4 GKGPU_LDS_HEAP=16 GKGPU_JIT_WPE=4
run h8w4 GKGPU_LDS_HEAP=8 GKGPU_JIT_WPE=4
