#!/bin/bash
# GPU diagnostics (run on the box from the repo root): GPU parity suite, the
# K8sContainerLimits cost breakdown by template variant, and the PMC counter list.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export GKGPU_JIT_CACHE=$PWD/.jitcache
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK
timeout -k 10 300 python -u tools/probe_variants.py 1000000 > gpurun_out/variants.log 2>&1 && echo VARIANTS_OK
cd /tmp && timeout -k 10 60 rocprofv3 -L > "$GRAFT_REPO_ROOT/gpurun_out/counters.txt" 2>&1; echo LIST_DONE
