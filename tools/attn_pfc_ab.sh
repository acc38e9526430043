#!/bin/bash
# Round 5: the attention's cells prefetched with the position (KQ_ATTN_PFC) 64 (product)
# against 128 (lib/variants/libpfc128.so), bench.py's headline token, three interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
FLAGS="--steps 128 --warmup 16 --no-cpu-baseline --no-large --no-prefill --no-chain --no-8b --no-70b --no-collectives --tg 0"
for r in 1 2 3; do
  for model in tinyllama-1.1b llama-3-8b; do
    for l in ${LIBS:-lib/libggml_mi355x.so lib/variants/libpfc128.so}; do
      MI355X_LIB=ggml-neon-opt_amd/$l timeout -k 10 300 python -u bench.py --model $model $FLAGS > gpurun_out/ab_tmp.json 2> gpurun_out/ab_tmp.err
      rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $l"; tail -5 gpurun_out/ab_tmp.err; exit $rc; }
      tail -1 gpurun_out/ab_tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r', '$model', '$l', d['value'], d['ms_per_step'])"
    done
  done
done
