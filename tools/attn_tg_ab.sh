#!/bin/bash
# Round 5: attention long-context A/B on one box: bench.py's tg side figure at 1024 and 20
# tokens for each library (product, variants), two interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBS=${LIBS:-"lib/libggml_mi355x.so lib/variants/libahead.so lib/variants/libakr2.so"}
for r in 1 2; do
  for l in $LIBS; do
    for n in ${TG_NS:-1024 20}; do
      MI355X_LIB=ggml-neon-opt_amd/$l timeout -k 10 300 python -u bench.py --steps 16 --warmup 4 --tg $n ${BENCH_EXTRA:-} > gpurun_out/ab_tmp.json 2> gpurun_out/ab_tmp.err
      rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $l $n"; tail -5 gpurun_out/ab_tmp.err; exit $rc; }
      tail -1 gpurun_out/ab_tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['tg128']; print('$r', '$l', '$n', t['tok_s'], t['tok_s_sd'])"
    done
  done
done
