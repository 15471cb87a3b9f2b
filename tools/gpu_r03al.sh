#!/bin/bash
# Short A/B of the function early exit on config 2 (GKGPU_FN_EARLY 0 / 1).
#   bash tools/gpu_r03al.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03al}
OUT=gpurun_out/$TAG
mkdir -p "$OUT" gpurun_out/jitcache
cp -n .jitcache/*.co gpurun_out/jitcache/ 2>/dev/null || true
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jitcache
for f in 0 1; do
  GKGPU_FN_EARLY=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-sample 0 > "$OUT/c2_e$f.json" 2> "$OUT/c2_e$f.err" || { echo "E${f}_FAIL"; tail "$OUT/c2_e$f.err"; exit 1; }
  python - "$OUT/c2_e$f.json" "c2 early=$f" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); c = d["config"]
ks = {c["kernel_templates"].get(k["kernel"], k["kernel"])[:16]: round(k["avg_ms"], 3) for k in d["kernels"]}
print("AB", sys.argv[2], round(d["value"] / 1e6, 1), round(d["ms_per_step"], 3), c["violations_per_step_rank0"], ks)
PY
done
