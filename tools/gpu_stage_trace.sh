#!/bin/bash
# staging trace of one config-2 bench run per storage form (GKGPU_COLUMNS)
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; mkdir -p "$OUT"
mkdir -p /tmp/gkjit_cache; cp -n .jitcache/*.co /tmp/gkjit_cache/ 2>/dev/null; export GKGPU_JIT_CACHE=/tmp/gkjit_cache
for v in 1 0; do
  GKGPU_COLUMNS=$v GKGPU_FLATTEN_TRACE=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 --shard-leg off > "$OUT/c2_$v.json" 2> "$OUT/c2_$v.err" || { echo FAIL; tail "$OUT/c2_$v.err"; exit 1; }
  echo "== cols $v"; grep -E "^columns|^upload|^stage|^flatten: (parse|intern|device)" "$OUT/c2_$v.err" | tail -14
done
