#!/bin/bash
# Round 5: GEMV remaining-work priority (stamps + token A/B) and kq_mmq static priority (prefill A/B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in diag diagp; do
  MI355X_LIB=ggml-neon-opt_amd/lib/variants/lib$v.so timeout -k 10 400 python -u tools/stamps.py rows > gpurun_out/r5s_stamps_$v.txt 2>&1 || exit $?
  echo $v; cut -c1-24,150-270 gpurun_out/r5s_stamps_$v.txt
done
MI355X_LIB= timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5s_ops_tests.log 2>&1 || { tail -20 gpurun_out/r5s_ops_tests.log; exit 1; }; tail -1 gpurun_out/r5s_ops_tests.log
bash tools/ab_libs.sh default prio > gpurun_out/r5s_ab_libs.txt 2>&1 || { tail -5 gpurun_out/r5s_ab_libs.txt; exit 1; }
tail -9 gpurun_out/r5s_ab_libs.txt | cut -c1-60
RUNS="tile128: tile128:mprio tile128: tile128:mprio" PREFILL_TYPES=12 bash tools/mmq_libs.sh > gpurun_out/r5s_mmq.txt 2>&1
tail -30 gpurun_out/r5s_mmq.txt
LIBS="lib/libggml_mi355x.so lib/variants/libaev0.so" bash tools/attn_tg_ab.sh > gpurun_out/r5s_attn_ab.txt 2>&1
cat gpurun_out/r5s_attn_ab.txt
