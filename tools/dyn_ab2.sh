#!/bin/bash
# Round 6: kq_rows_dyn placements A/B: static split (GEMV_DYN=0), claimed units strided over
# the matrix (product build), claimed units from one contiguous row range (variant dyncontig).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$PWD/ggml-neon-opt_amd/lib/variants
OUT=gpurun_out/dyn_ab2.txt
: > $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -x -q -k "dyn" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/dyn_ab2_tests0.log 2>&1 || { tail -20 gpurun_out/dyn_ab2_tests0.log; exit 1; }
MI355X_LIB=$V/libdyncontig.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "dyn" \
   --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/dyn_ab2_tests.log 2>&1 || { tail -20 gpurun_out/dyn_ab2_tests.log; exit 1; }
for r in 1 2; do
  for cfg in static strided contig; do
    echo "== large $cfg (round $r)" >> $OUT
    unset MI355X_LIB MI355X_GEMV_DYN
    [ $cfg = static ] && export MI355X_GEMV_DYN=0
    [ $cfg = contig ] && export MI355X_LIB=$V/libdyncontig.so
    timeout -k 10 150 python -u tools/gemv_large_ab.py 2>&1 | grep -v amdgpu.ids >> $OUT || exit $?
  done
done
unset MI355X_LIB MI355X_GEMV_DYN
MODELS="llama-3-8b" KNOBSETS="- GEMV_DYN=0" timeout -k 10 600 bash tools/knob_ab.sh >> $OUT 2>&1 || exit $?
cat $OUT
