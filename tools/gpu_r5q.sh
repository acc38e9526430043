#!/bin/bash
# Round 5: the split attention at long caches: TinyLlama tg at TG_NS cells (default 2048) for
# the product, the build before the early chunk (aprev) and the per-head kernel (ahead);
# PARITY=1 runs the attention parity tests first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${PARITY:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -k "attn" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5q_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/r5q_tests.log; [ $rc -eq 0 ] || exit $rc
fi
LIBS="lib/libggml_mi355x.so lib/variants/libaprev.so lib/variants/libahead.so" TG_NS="${TG_NS:-2048}" timeout -k 10 900 bash tools/attn_tg_ab.sh
