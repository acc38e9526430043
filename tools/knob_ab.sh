#!/bin/bash
# Round 5: bench.py's headline token (TinyLlama and Llama-3-8B) under experiment knobs
# (--knob NAME=V, the library's A/B knobs), three interleaved rounds.
#   KNOBSETS="- GEMV_SMALL_WG=128 GEMV_SMALL_WG=192": one variant per word, "-" = product,
#   several knobs in one variant joined by commas
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
FLAGS="--steps 128 --warmup 16 --no-cpu-baseline --no-large --no-prefill --no-chain --no-8b --no-70b --no-collectives --tg 0"
for r in 1 2 3; do
  for model in ${MODELS:-tinyllama-1.1b llama-3-8b}; do
    for ks in ${KNOBSETS:--}; do
      kargs=""
      [ "$ks" = "-" ] || for k in ${ks//,/ }; do kargs="$kargs --knob $k"; done
      timeout -k 10 300 python -u bench.py --model $model $FLAGS $kargs > gpurun_out/ab_tmp.json 2> gpurun_out/ab_tmp.err
      rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $ks"; tail -5 gpurun_out/ab_tmp.err; exit $rc; }
      tail -1 gpurun_out/ab_tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r', '$model', '$ks', d['value'], d['ms_per_step'])"
    done
  done
done
