#!/bin/bash
# Round 5: attention K-ring depth (KQ_ATTN_KD=3 variant): parity on the variant, then tg A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VAR=${VAR_LIB:-ggml-neon-opt_amd/lib/variants/libakd3.so}
MI355X_LIB=$VAR timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "attn" -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r5y_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5y_tests.log; [ $rc -eq 0 ] || exit $rc
LIBS=${TG_LIBS:-"lib/libggml_mi355x.so lib/variants/libakd3.so"} timeout -k 10 900 bash tools/attn_tg_ab.sh
