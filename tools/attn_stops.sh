#!/bin/bash
# Where kq_attn_decode's replayed time goes: the TinyLlama token under rocprofv3 kernel trace
# with the diagnostic build (lib/variants/libadiag.so, make variant-ops NAME=adiag
# VFLAGS=-DKQ_ATTN_DIAG=1) stopped at each MI355X_ATTN_DIAG point: 4 empty launch, 5 loads
# without the KV cache + rope, 1 loads + rope, 2 + KQ, 3 + soft_max, 0 complete.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/attn_stops
mkdir -p $OUT
for d in 4 5 1 2 3 0; do
  MI355X_LIB=$PWD/ggml-neon-opt_amd/lib/variants/libadiag.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
      --output-format csv -d $OUT/d$d -o run -- python3 bench.py --steps 64 --warmup 8 --no-cpu-baseline --no-large \
      --no-prefill --no-8b --no-70b --no-chain --tg 0 --no-collectives --knob ATTN_DIAG=$d > $OUT/d$d.log 2>&1 || exit $?
  python3 - $OUT/d$d/run_kernel_stats.csv $d <<'PY' || exit $?
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "attn_decode" in r["Name"]:
        print("diag", sys.argv[2], r["Name"][:40], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 3), flush=True)
PY
  rm -f $OUT/d$d/run_kernel_trace.csv
  grep -o '"value": [0-9.]*' $OUT/d$d.log | head -1
done
# the same stops without the profiler: token time with an empty attention against the product build
for d in 4 0; do
  MI355X_LIB=$PWD/ggml-neon-opt_amd/lib/variants/libadiag.so timeout -k 10 200 python3 bench.py --steps 64 --warmup 8 \
      --no-cpu-baseline --no-large --no-prefill --no-8b --no-70b --no-chain --tg 0 --no-collectives --knob ATTN_DIAG=$d \
      > $OUT/plain_d$d.log 2>&1 || exit $?
  echo "plain diag $d $(grep -o '"value": [0-9.]*' $OUT/plain_d$d.log | head -1)"
done
