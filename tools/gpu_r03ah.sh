#!/bin/bash
# A/B, one call, alternating: review order largest-first (GKGPU_ORDER_DESC=1)
# on configs 2 and 4, and the dword-gathering format writer
# (GKGPU_FMT_WORDS=1) on config 2; then message parity with the latter.
#   bash tools/gpu_r03ah.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03ah}
OUT=gpurun_out/$TAG
mkdir -p "$OUT" gpurun_out/jitcache
cp -n .jitcache/*.co gpurun_out/jitcache/ 2>/dev/null || true
export GKGPU_JIT_CACHE=$PWD/gpurun_out/jitcache
run() {  # name cfg env...
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 400 python -u bench.py --config $cfg --steps 20 --warmup 3 --cpu-sample 0 > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "${name}_FAIL"; tail "$OUT/$name.err"; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); c = d["config"]
ks = {c["kernel_templates"].get(k["kernel"], k["kernel"])[:16]: round(k["avg_ms"], 3) for k in d["kernels"]}
print("AB", sys.argv[2], round(d["value"] / 1e6, 1), round(d["ms_per_step"], 3), ks)
PY
}
for rep in 1 2; do
  run c2_base_$rep 2 GKGPU_ORDER_DESC=0 && run c2_desc_$rep 2 GKGPU_ORDER_DESC=1 && run c2_words_$rep 2 GKGPU_FMT_WORDS=1 && \
  run c4_base_$rep 4 GKGPU_ORDER_DESC=0 && run c4_desc_$rep 4 GKGPU_ORDER_DESC=1 || exit 1
done
GKGPU_FMT_WORDS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread \
  -k "config2_agilebank_pods or psp_object_printing or config5 or output_buffers" > "$OUT/pytest_words.log" 2>&1
rc=$?
tail -2 "$OUT/pytest_words.log"
exit $rc
