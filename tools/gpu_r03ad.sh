#!/bin/bash
# Sampling passes after the wave-aggregated histogram: the audit / sampling /
# device-output tests, then the default bench (config 2).
#   bash tools/gpu_r03ad.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03ad}
OUT=gpurun_out/$TAG
mkdir -p "$OUT" gpurun_out/jitcache
cp -n .jitcache/*.co gpurun_out/jitcache/ 2>/dev/null || true
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -v --timeout 300 \
  --timeout-method thread -k "audit or sample or device_output" > "$OUT/sample_tests.log" 2>&1
rc=$?
tail -3 "$OUT/sample_tests.log"
[ $rc -eq 0 ] || { echo TESTS_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-sample 0 > "$OUT/c2.json" 2> "$OUT/c2.err" || { echo BENCH_FAIL; tail "$OUT/c2.err"; exit 1; }
python - "$OUT/c2.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
ks = d["roofline"].get("kernels") or []
print(round(d["value"] / 1e6, 1), round(d["ms_per_step"], 3), [(k["kernel"][:14], round(k["avg_ms"], 3)) for k in ks])
PY
