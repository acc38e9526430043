#!/bin/bash
# Attention: parity of the product build (early post-position K/V loads), the token A/B against
# the previous attention builds (lib/variants/libearly0.so: KQ_ATTN_EARLY=0; libpf0.so: every
# cell prefetched with the position, round 3), and the plain (unprofiled) stops of the
# diagnostic build (lib/variants/libadiag.so, finite stop outputs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$PWD/ggml-neon-opt_amd/lib/variants
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_attn_oproj.py -x -q -k "attn or llama" \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04j_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04j_tests.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=2 timeout -k 10 900 bash tools/ab_ao.sh tiny 8b tiny,lib:early0 8b,lib:early0 tiny,lib:pf0 8b,lib:pf0 || exit $?
cp gpurun_out/ab_ao.log gpurun_out/r04j_attn_ab.log
: > gpurun_out/r04j_stops.log
for r in 1 2; do
  for d in 4 5 1 2 3 0; do
    MI355X_LIB=$V/libadiag.so timeout -k 10 200 python3 bench.py --steps 64 --warmup 8 --no-cpu-baseline --no-large \
        --no-prefill --no-8b --no-70b --no-chain --tg 0 --no-collectives --knob ATTN_DIAG=$d > gpurun_out/stop.json 2>&1 || exit $?
    echo "diag $d $(grep -o '"value": [0-9.]*' gpurun_out/stop.json | head -1)" | tee -a gpurun_out/r04j_stops.log
  done
done
