#!/bin/bash
# The 10M-resource config-4 sweep (tools/sweep_10m.py: 64-bit outputs + sampled
# parity), then bench lines for configs 3, 4 and 5 at HEAD.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02f
export GKGPU_JIT_CACHE=$PWD/.jitcache
rocm-smi --showclocks > gpurun_out/r02f/clocks_before.txt 2>&1 || true
timeout -k 10 300 python -u tools/sweep_10m.py 200000 200 > gpurun_out/r02f/sweep_small.log 2>&1 || { tail -20 gpurun_out/r02f/sweep_small.log; exit 1; }
tail -1 gpurun_out/r02f/sweep_small.log
timeout -k 10 900 python -u tools/sweep_10m.py 10000000 600 > gpurun_out/r02f/sweep_10m.log 2>&1 || { tail -20 gpurun_out/r02f/sweep_10m.log; exit 1; }
tail -1 gpurun_out/r02f/sweep_10m.log
for c in 3 4 5; do
  timeout -k 10 600 python -u bench.py --config $c > gpurun_out/r02f/bench_config$c.json 2> gpurun_out/r02f/bench_config$c.err || { tail -20 gpurun_out/r02f/bench_config$c.err; exit 1; }
  echo "config $c: $(tail -1 gpurun_out/r02f/bench_config$c.json | cut -c1-300)"
done
rocm-smi --showclocks > gpurun_out/r02f/clocks_after.txt 2>&1 || true
