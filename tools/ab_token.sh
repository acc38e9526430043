#!/bin/bash
# Token-bench A/B over library variants, interleaved twice (bench line only).
# usage (GPU box): bash tools/ab_token.sh default ggml-neon-opt_amd/lib/variants/libX.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/ab_token.log
: > $OUT
for round in 1 2; do
  for L in "$@"; do
    if [ "$L" = default ]; then unset MI355X_LIB; else export MI355X_LIB=$PWD/$L; fi
    timeout -k 10 200 python bench.py --steps 64 --warmup 8 --no-cpu-baseline --no-large --no-prefill --no-8b --no-70b --no-chain --tg 0 ${BENCH_ARGS:-} > gpurun_out/ab_one.json 2>/dev/null || exit $?
    python - "$L" >> $OUT <<'PY' || exit $?
import json, sys
d = json.loads(open("gpurun_out/ab_one.json").read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], d["value"], d["ms_per_step"], {k.replace("kq::", ""): v["us_per_launch"] for k, v in d["kernels"].items()}, flush=True)
PY
  done
done
cat $OUT
