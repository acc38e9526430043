#!/bin/bash
# Round 6: long-cache decode attention, KQ split over cells (two launches, product) against the
# one-workgroup-per-head kernel (variant nocells): the attention GPU tests, then bench.py's tg
# side figure at 4096 / 2048 / 20 tokens (positions 0..n-1 of a fresh cache), two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "attn" --timeout 200 --timeout-method thread \
   -p no:cacheprovider > gpurun_out/cells_tests.log 2>&1 || { tail -30 gpurun_out/cells_tests.log; exit 1; }
tail -2 gpurun_out/cells_tests.log
OUT=gpurun_out/cells_ab.txt
: > $OUT
for r in 1 2; do
  for l in ${LIBS:-lib/libggml_mi355x.so lib/variants/libnocells.so}; do
    for n in ${TG_NS:-4096 2048 20}; do
      MI355X_LIB=ggml-neon-opt_amd/$l timeout -k 10 300 python -u bench.py --steps 16 --warmup 4 --tg $n --no-cpu-baseline \
          --no-large --no-prefill --no-chain --no-8b --no-70b --no-collectives ${BENCH_EXTRA:-} > gpurun_out/ab_tmp.json 2> gpurun_out/ab_tmp.err
      rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $l $n"; tail -5 gpurun_out/ab_tmp.err; exit $rc; }
      tail -1 gpurun_out/ab_tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['tg128']; print('$r', '$l', '$n', t['tok_s'], t.get('tok_s_sd'))" >> $OUT
    done
  done
done
cat $OUT
