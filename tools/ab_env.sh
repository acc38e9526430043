#!/bin/bash
# Token-bench A/B over environment settings, interleaved twice (bench line only).
# usage (GPU box): bash tools/ab_env.sh "A=1 B=2" "A=0" ...   (one quoted env set per variant; "" = default)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/ab_env.log
: > $OUT
for round in $(seq ${ROUNDS:-2}); do
  for E in "$@"; do
    env $E timeout -k 10 200 python bench.py --steps 64 --warmup 8 --no-cpu-baseline --no-large --no-prefill --no-8b --no-70b --no-chain --no-collectives --tg 0 ${BENCH_ARGS:-} > gpurun_out/ab_one.json 2>/dev/null || exit $?
    python - "$E" >> $OUT <<'PY' || exit $?
import json, sys
d = json.loads(open("gpurun_out/ab_one.json").read().strip().splitlines()[-1])
print(repr(sys.argv[1]), d["value"], d["ms_per_step"], {k.replace("kq::", ""): v["us_per_launch"] for k, v in d["kernels"].items()}, flush=True)
PY
  done
done
cat $OUT
