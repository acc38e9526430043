#!/bin/bash
# Round 6: the context curve's crossover between the output split and the split over cells:
# tg at n tokens on each library of LIBS, TinyLlama (TINY_NS) and Llama-3-8B (B8_NS).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/ctx_ab.txt
: > $OUT
run() {  # lib[:KNOB=V] model n
  local lib=${1%%:*} kn=""
  [ "$lib" != "$1" ] && kn="--knob ${1#*:}" && kn=${kn//,/ --knob }  # lib:K1=V1,K2=V2
  MI355X_LIB=ggml-neon-opt_amd/$lib timeout -k 10 400 python -u bench.py --model $2 --steps 16 --warmup 4 --tg $3 --no-cpu-baseline --no-large \
      --no-prefill --no-chain --no-8b --no-70b --no-collectives $kn > gpurun_out/cc_tmp.json 2> gpurun_out/cc_tmp.err
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $1 $2 $3"; tail -5 gpurun_out/cc_tmp.err; exit $rc; }
  tail -1 gpurun_out/cc_tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['tg128']; print('$1', '$2', '$3', t['tok_s'], t.get('tok_s_sd'))" | tee -a $OUT
}
for l in ${LIBS}; do
  for n in ${TINY_NS:-}; do run $l tinyllama-1.1b $n; done
  for n in ${B8_NS:-}; do run $l llama-3-8b $n; done
  for n in ${B70_NS:-}; do run $l llama-3-70b $n; done
done
cat $OUT
