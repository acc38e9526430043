#!/bin/bash
# Round 5: attention heads split by output over 4 / 8 workgroups past 256 cache cells
# (MI355X_ATTN_SPLIT): parity of every attention kernel, launch timings, tg A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_attn_oproj.py tests/test_gpu_layer.py -k "attn or layer" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5w_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5w_tests.log; [ $rc -eq 0 ] || exit $rc
PREV=${PREV_LIB:-ggml-neon-opt_amd/lib/variants/libaprev.so}
for rr in 1 0; do
  echo "== rope_row=$rr head"; ATTN_PHASES_ROPE_ROW=$rr MI355X_ATTN_IMPL=head ATTN_PHASES_DIAGS=0 timeout -k 10 300 python -u tools/attn_phases.py || exit $?
  echo "== rope_row=$rr split"; ATTN_PHASES_ROPE_ROW=$rr MI355X_ATTN_IMPL=split ATTN_PHASES_DIAGS=0 timeout -k 10 300 python -u tools/attn_phases.py || exit $?
  echo "== rope_row=$rr split prev"; MI355X_LIB=$PREV ATTN_PHASES_ROPE_ROW=$rr MI355X_ATTN_IMPL=split ATTN_PHASES_DIAGS=0 timeout -k 10 300 python -u tools/attn_phases.py || exit $?
done
LIBS=${TG_LIBS:-"lib/libggml_mi355x.so lib/variants/libaprev.so lib/variants/libahead.so"} timeout -k 10 900 bash tools/attn_tg_ab.sh
