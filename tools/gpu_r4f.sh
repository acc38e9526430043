#!/bin/bash
# The fused attention + o-proj kernel's parity tests on the current build and the attention
# parity tests on the prefetch-bound builds (lib/variants/libpf32/64.so), then the token A/B
# (tools/ab_ao.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$PWD/ggml-neon-opt_amd/lib/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_attn_oproj.py -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r04f_ao_tests.log 2>&1
rc=$?; echo "ao tests rc=$rc"; tail -3 gpurun_out/r04f_ao_tests.log
[ $rc -eq 0 ] || exit $rc
for L in pf32 pf64; do
  MI355X_LIB=$V/lib$L.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "attn or llama" --timeout 120 \
      --timeout-method thread -p no:cacheprovider > gpurun_out/r04f_${L}_tests.log 2>&1
  rc=$?; echo "$L tests rc=$rc"; tail -2 gpurun_out/r04f_${L}_tests.log
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 1000 bash tools/ab_ao.sh tiny 8b tiny,knob:ATTN_OPROJ=0 8b,knob:ATTN_OPROJ=0 tiny,knob:AO_NRB=16 \
    tiny,lib:ao1 tiny,lib:ao2 tiny,lib:ao4 tiny,lib:pf32,knob:ATTN_OPROJ=0 tiny,lib:pf64,knob:ATTN_OPROJ=0
