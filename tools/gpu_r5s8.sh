#!/bin/bash
# Round 5: 8 instead of 6 waves per workgroup for decode GEMVs under 10 MB (variant ws8:
# TinyLlama's 2048-row matrices get exactly one row per wave): GEMV parity on the variant,
# then decode tokens, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
MI355X_LIB=ggml-neon-opt_amd/lib/variants/libws8.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ops.py -k "gemv or llama_decode" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5s8_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5s8_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for lib in lib/libggml_mi355x.so lib/variants/libws8.so; do
    for m in tinyllama-1.1b llama-3-8b; do
      MI355X_LIB=ggml-neon-opt_amd/$lib timeout -k 10 300 python -u bench.py --model $m --steps 64 --warmup 8 --tg 0 --no-70b --no-8b --no-large --no-prefill --no-chain --no-collectives --no-cpu-baseline > gpurun_out/s8_tmp.json 2> gpurun_out/s8_tmp.err
      rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/s8_tmp.err; exit $rc; }
      tail -1 gpurun_out/s8_tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r $lib $m', d['value'], d['step_ms']['p50'])"
    done
  done
done
