#!/bin/bash
# A/B on one box: bench (and a GEMV sweep) for each library given, interleaved twice.
# usage (on the GPU box): bash tools/ab.sh default ggml-neon-opt_amd/lib/variants/libX.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/ab.log
: > $OUT
for round in 1 2; do
  for L in "$@"; do
    if [ "$L" = default ]; then unset MI355X_LIB; else export MI355X_LIB=$PWD/$L; fi
    echo "== round $round lib=$L" >> $OUT
    timeout -k 10 300 python bench.py --steps 64 --warmup 8 --no-cpu-baseline --no-large 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], {k: v['us_per_launch'] for k, v in d['kernels'].items()})" >> $OUT || exit $?
    if [ $round = 1 ]; then timeout -k 10 300 python tools/gemv_sweep.py auto >> $OUT 2>&1 || exit $?; fi
  done
done
cat $OUT
