#!/bin/bash
# A/B of the review order: ascending document size (default) against largest
# first (GKGPU_ORDER_DESC=1), configs 2 and 4, alternating, one call.
#   bash tools/gpu_r03ah.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03ah}
OUT=gpurun_out/$TAG
mkdir -p "$OUT" gpurun_out/jitcache
cp -n .jitcache/*.co gpurun_out/jitcache/ 2>/dev/null || true
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jitcache
for rep in 1 2; do
  for cfg in 2 4; do
    for d in 0 1; do
      GKGPU_ORDER_DESC=$d timeout -k 10 400 python -u bench.py --config $cfg --steps 20 --warmup 3 --cpu-sample 0 > "$OUT/c${cfg}_d${d}_$rep.json" 2> "$OUT/c${cfg}_d${d}_$rep.err" || { echo "C${cfg}_D${d}_FAIL"; tail "$OUT/c${cfg}_d${d}_$rep.err"; exit 1; }
      python - "$OUT/c${cfg}_d${d}_$rep.json" "c${cfg} desc=$d rep $rep" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); c = d["config"]
ks = {c["kernel_templates"].get(k["kernel"], k["kernel"])[:16]: round(k["avg_ms"], 3) for k in d["kernels"]}
print(sys.argv[2], round(d["value"] / 1e6, 1), round(d["ms_per_step"], 3), ks)
PY
    done
  done
done
