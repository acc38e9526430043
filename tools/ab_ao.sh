#!/bin/bash
# A/B of the attention + o-proj fusion (kq_attn_oproj) on one box, interleaved twice:
# the product, fusion off (knob ATTN_OPROJ=0), row-block counts (knob AO_NRB) and the
# timing ablations of `make variant-ao` (lib/variants/libaoN.so: 1 no attention, 2 stop
# after the attention, 4 no hand-off, 8 no weight DMA), TinyLlama and Llama-3-8B tokens.
#   usage (GPU box): bash tools/ab_ao.sh [CONFIG...]   CONFIG: default | knob:NAME=V | lib:NAME
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$PWD/ggml-neon-opt_amd/lib/variants
CFGS=("$@")
[ ${#CFGS[@]} -eq 0 ] && CFGS=(default knob:ATTN_OPROJ=0 knob:AO_NRB=8 knob:AO_NRB=16 lib:ao1 lib:ao2 lib:ao4 lib:ao8)
OUT=gpurun_out/ab_ao.log
: > $OUT
for r in 1 2; do
  for C in "${CFGS[@]}"; do
    for model in tinyllama-1.1b llama-3-8b; do
      unset MI355X_LIB
      EXTRA=""
      case $C in
        knob:*) EXTRA="--knob ${C#knob:}" ;;
        lib:*) export MI355X_LIB=$V/lib${C#lib:}.so ;;
      esac
      timeout -k 10 200 python bench.py --model $model --steps 64 --warmup 8 --no-cpu-baseline --no-large \
          --no-prefill --no-8b --no-70b --no-chain --tg 0 --no-collectives $EXTRA > gpurun_out/ab_one.json 2>gpurun_out/ab_one.err || exit $?
      python - "$C $model" >> $OUT <<'PY' || exit $?
import json, sys
d = json.loads(open("gpurun_out/ab_one.json").read().strip().splitlines()[-1])
k = {n.replace("kq::", ""): v["us_per_launch"] for n, v in d["kernels"].items() if "attn" in n or "<1, true, 0>" in n}
print(sys.argv[1], d["value"], d["ms_per_step"], d["config"]["stages_per_token"], k, flush=True)
PY
      tail -1 $OUT
    done
  done
done
unset MI355X_LIB
