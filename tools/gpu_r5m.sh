#!/bin/bash
# Round 5: the 128 x 64 prefill tile for 128 x 128 grids that fill under 384 workgroups:
# parity (mmq + prompt tests), then eager prompt per-kernel sums against the previous rule
# (mprev), TinyLlama and Llama-3-8B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -k "prompt or mmq" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5m_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5m_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for lib in lib/libggml_mi355x.so lib/variants/libmprev.so; do
    for m in tinyllama-1.1b llama-3-8b; do
      echo "== $r $lib $m"
      MI355X_LIB=ggml-neon-opt_amd/$lib timeout -k 10 200 python3 tools/prompt_profile.py $m 2>/dev/null | grep -E "kq_mmq|total" || exit 1
    done
  done
done
