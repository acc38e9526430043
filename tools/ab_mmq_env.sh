#!/bin/bash
# Prefill A/B over MI355X_MMQ_IMPL (auto / k4 / tile64): TinyLlama and Llama-3-8B pp512 through
# the prompt graph, interleaved ROUNDS times. usage (GPU box): bash tools/ab_mmq_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/ab_mmq.log
: > $OUT
for round in $(seq ${ROUNDS:-2}); do
  for E in "" "MI355X_MMQ_IMPL=tile64"; do
    env $E timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-large --no-chain --no-70b --tg 0 > gpurun_out/ab_mmq_one.json 2>/dev/null || exit $?
    python - "$E" >> $OUT <<'PY' || exit $?
import json, sys
d = json.loads(open("gpurun_out/ab_mmq_one.json").read().strip().splitlines()[-1])
b = d.get("llama3_8b") or {}
print(repr(sys.argv[1]), "tiny pp512", (d.get("pp512") or {}).get("ms_per_batch"),
      "| 8B pp512 graph", (b.get("pp512_graph") or {}).get("ms_per_batch"), flush=True)
PY
  done
done
cat $OUT
