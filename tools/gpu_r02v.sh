#!/bin/bash
# Inventory-join parity (both back ends), stage-upload trace, and the
# two-rank bench path rehearsed on one GPU over gloo.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02v
export GKGPU_JIT_CACHE=$PWD/.jitcache
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread -k "unique_service" > gpurun_out/r02v/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r02v/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
GKGPU_FLATTEN_TRACE=1 timeout -k 10 300 python -u bench.py --cpu-sample 0 --steps 5 > gpurun_out/r02v/bench1.json 2> gpurun_out/r02v/bench1.err || exit 1
grep -h "sync_tables\|upload" gpurun_out/r02v/bench1.err
GKGPU_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --cpu-sample 0 --pods 500000 > gpurun_out/r02v/bench2.json 2> gpurun_out/r02v/bench2.err || { echo "gloo rehearsal failed"; tail -20 gpurun_out/r02v/bench2.err; exit 1; }
tail -c 1500 gpurun_out/r02v/bench2.json
exit $rc
