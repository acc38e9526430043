#!/bin/bash
# Headline sensitivity to --steps / --warmup (token workload only, no side figures).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; OUT=gpurun_out/steps_probe.log; : > $OUT
for sw in "20 5" "20 5" "20 30" "128 5" "20 5"; do
  set -- $sw
  timeout -k 10 120 python bench.py --steps $1 --warmup $2 --no-cpu-baseline --no-large --no-prefill --no-8b --no-70b --no-chain --tg 128 > gpurun_out/sp.json 2>/dev/null || exit $?
  python - "$sw" >> $OUT <<'PY'
import json, sys
d = json.loads(open("gpurun_out/sp.json").read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], d["ms_per_step"], d["gpu_ms_per_step"], d["tg128"]["ms_per_token"], flush=True)
PY
done
cat $OUT
