#!/bin/bash
# Decode-token A/B on one box, interleaved ROUNDS times: the product, the attention + o-proj
# fusion forced on (knob ATTN_OPROJ=2; the product leaves it off), row-block counts (knob AO_NRB), the timing ablations of
# `make variant-ao` (lib/variants/libaoN.so: 1 no attention, 2 stop after the attention,
# 4 no hand-off, 8 no weight DMA) and other variant builds.
#   usage (GPU box): bash tools/ab_ao.sh [CONFIG...]
#   CONFIG: MODEL[,lib:NAME][,knob:NAME=V]...   MODEL: tiny | 8b
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$PWD/ggml-neon-opt_amd/lib/variants
CFGS=("$@")
[ ${#CFGS[@]} -eq 0 ] && CFGS=(tiny 8b tiny,knob:ATTN_OPROJ=2 8b,knob:ATTN_OPROJ=2 tiny,knob:ATTN_OPROJ=2,knob:AO_NRB=16 tiny,lib:ao1,knob:ATTN_OPROJ=2
                              tiny,lib:ao2,knob:ATTN_OPROJ=2 tiny,lib:ao4,knob:ATTN_OPROJ=2 tiny,lib:ao8,knob:ATTN_OPROJ=2)
OUT=gpurun_out/ab_ao.log
: > $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for C in "${CFGS[@]}"; do
    unset MI355X_LIB
    EXTRA=""
    model=tinyllama-1.1b
    IFS=, read -ra parts <<< "$C"
    for p in "${parts[@]}"; do
      case $p in
        tiny) model=tinyllama-1.1b ;;
        8b) model=llama-3-8b ;;
        knob:*) EXTRA="$EXTRA --knob ${p#knob:}" ;;
        lib:*) export MI355X_LIB=$V/lib${p#lib:}.so ;;
      esac
    done
    timeout -k 10 200 python bench.py --model $model --steps 64 --warmup 8 --no-cpu-baseline --no-large \
        --no-prefill --no-8b --no-70b --no-chain --tg 0 --no-collectives $EXTRA > gpurun_out/ab_one.json 2>gpurun_out/ab_one.err || exit $?
    python - "$C" >> $OUT <<'PY' || exit $?
import json, sys
d = json.loads(open("gpurun_out/ab_one.json").read().strip().splitlines()[-1])
k = {n.replace("kq::", ""): v["us_per_launch"] for n, v in d["kernels"].items() if "attn" in n or "<1, true, 0>" in n}
print(sys.argv[1], d["value"], d["ms_per_step"], d["config"]["stages_per_token"], k, flush=True)
PY
    tail -1 $OUT
  done
done
unset MI355X_LIB
