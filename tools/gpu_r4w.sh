#!/bin/bash
# Llama-3-8B pp512 (matmul chain + prompt graph) on the product (packed Q4_K chain) vs
# lib/variants/libpk0.so (KQ_MMQ_PKCHAIN=0), interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/r04w_pp.log
for r in 1 2; do
  for L in product pk0; do
    lib=""; [ $L != product ] && lib=$PWD/ggml-neon-opt_amd/lib/variants/lib$L.so
    MI355X_LIB=$lib timeout -k 10 300 python bench.py --model llama-3-8b --steps 16 --warmup 4 --no-cpu-baseline --no-large \
        --no-70b --no-chain --no-8b --tg 0 --no-collectives > gpurun_out/pp.json 2>&1 || exit $?
    python3 - "$L" >> gpurun_out/r04w_pp.log <<'PY' || exit $?
import json, sys
d = json.loads([l for l in open("gpurun_out/pp.json") if l.startswith("{")][-1])
p = d["prefill_pp512"]
print(sys.argv[1], "matmuls", p.get("ms"), "ms", p.get("int_TOPS"), "TOPS", "graph", (d.get("pp512") or {}).get("ms"), "ms",
      {k: v["us_per_launch"] for k, v in (p.get("kernels") or {}).items()} if isinstance(p.get("kernels"), dict) else "", flush=True)
PY
    tail -1 gpurun_out/r04w_pp.log
  done
done
