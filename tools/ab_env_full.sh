#!/bin/bash
# A/B of environment settings on the token (tg20 headline + tg128) and the TinyLlama pp512,
# interleaved twice; one line per run. usage: bash tools/ab_env_full.sh "" "A=1" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/ab_env_full.log
: > $OUT
for round in 1 2; do
  for E in "$@"; do
    env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-large --no-8b --no-70b --no-chain --tg 128 > gpurun_out/ab_one.json 2>/dev/null || exit $?
    python - "$E" >> $OUT <<'PY' || exit $?
import json, sys
d = json.loads(open("gpurun_out/ab_one.json").read().strip().splitlines()[-1])
print(repr(sys.argv[1]), "tg20", d["ms_per_step"], "tg128", d["tg128"]["ms_per_token"], "pp512", d["prefill_pp512"]["ms_per_batch"],
      {k.replace("kq::", ""): v["us_per_launch"] for k, v in d["kernels"].items() if "attn" in k}, flush=True)
PY
  done
done
cat $OUT
