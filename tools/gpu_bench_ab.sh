#!/bin/bash
# Same-call A/B of engine switches on one bench workload: bench.py once per
# setting (one process each), then one summary line per run (evals/s, ms/step,
# violations, per-template kernel ms).
#   bash tools/gpu_bench_ab.sh <tag> "<bench args>" "<setting>" ["<setting>" ...]
#   (setting: "" for the defaults, or "VAR=val VAR2=val")
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; BARGS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
# (gpu_measure.sh / gpu_final.sh set GKGPU_JIT_CACHE; standalone: seeded from .jitcache)
if [ -z "$GKGPU_JIT_CACHE" ]; then mkdir -p /tmp/gkjit_cache; cp -n .jitcache/*.co /tmp/gkjit_cache/ 2>/dev/null || true; export GKGPU_JIT_CACHE=/tmp/gkjit_cache; fi
i=0
for s in "$@"; do
  i=$((i+1))
  env $s timeout -k 10 400 python -u bench.py $BARGS --cpu-sample 0 > "$OUT/ab$i.json" 2> "$OUT/ab$i.err" || { echo "AB_FAIL [$i] $s"; tail "$OUT/ab$i.err"; exit 1; }
  python - "$OUT/ab$i.json" "[$i] ${s:-default}" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c = d["config"]
ks = {c["kernel_templates"].get(k["kernel"], k["kernel"])[:18]: round(k["avg_ms"], 3) for k in d["kernels"]}
print("AB", sys.argv[2], round(d["value"] / 1e6, 1), "M/s", round(d["ms_per_step"], 3), "ms", c["violations_per_step_rank0"],
      "viol", c["fallback_reviews"], "fb", ks, flush=True)
PY
done
