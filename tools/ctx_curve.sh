#!/bin/bash
# Round 6: decode tokens/s over context (bench.py's tg side figure at n tokens: positions 0..n-1
# of a fresh cache), TinyLlama and Llama-3-8B, on the product library (MI355X_LIB to compare).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/ctx_curve.txt
: > $OUT
run() {  # model n
  timeout -k 10 400 python -u bench.py --model $1 --steps 16 --warmup 4 --tg $2 --no-cpu-baseline --no-large \
      --no-prefill --no-chain --no-8b --no-70b --no-collectives > gpurun_out/cc_tmp.json 2> gpurun_out/cc_tmp.err
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $1 $2"; tail -5 gpurun_out/cc_tmp.err; exit $rc; }
  tail -1 gpurun_out/cc_tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['tg128']; print('$1', '$2', t['tok_s'], t.get('tok_s_sd'))" | tee -a $OUT
}
for n in ${TINY_NS:-20 512 1024 2048 3072 4096}; do run tinyllama-1.1b $n; done
for n in ${B8_NS:-20 1024 2048 4096}; do run llama-3-8b $n; done
cat $OUT
