#!/bin/bash
# Round 5: the head_dim-128 K ring (lane pairs) of the split attention: parity, phases, the
# Llama-3-8B tg at 512 / 20 cells and the TinyLlama tg1024 A/B against the previous build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_attn_oproj.py tests/test_gpu_layer.py -k "attn or layer" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5z_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5z_tests.log; [ $rc -eq 0 ] || exit $rc
for lib in lib/libggml_mi355x.so lib/variants/libaprev.so; do
  echo "== $lib"; MI355X_LIB=ggml-neon-opt_amd/$lib ATTN_PHASES_ROPE_ROW=1 ATTN_PHASES_DIAGS=0 timeout -k 10 300 python -u tools/attn_phases.py || exit $?
done
LIBS="lib/libggml_mi355x.so lib/variants/libaprev.so" TG_NS="512 20" BENCH_EXTRA="--model llama-3-8b --no-70b --no-8b --no-large --no-prefill --no-chain --no-collectives --no-cpu-baseline" timeout -k 10 900 bash tools/attn_tg_ab.sh || exit $?
LIBS="lib/libggml_mi355x.so lib/variants/libaprev.so" timeout -k 10 900 bash tools/attn_tg_ab.sh
