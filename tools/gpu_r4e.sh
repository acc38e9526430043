#!/bin/bash
# Prefill: the 3-buffer kq_mmq experiment build (lib/variants/libnb3.so: KQ_MMQ_NBUF=3 on the
# one-workgroup-per-CU tiles) — its prefill parity tests, then the prefill shapes on the product
# and on nb3 interleaved twice, then the MFMA PMC pass of the shipping kernels (tools/prof_prefill.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MI355X_LIB=$PWD/ggml-neon-opt_amd/lib/variants/libnb3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_ops.py -x -q -k "mmq or prefill or prompt or batch" --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r04e_nb3_tests.log 2>&1
rc=$?; echo "nb3 tests rc=$rc"; tail -3 gpurun_out/r04e_nb3_tests.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/r04e_mmq_ab.log
for r in 1 2; do
  for L in product nb3; do
    lib=""; [ $L != product ] && lib=$PWD/ggml-neon-opt_amd/lib/variants/lib$L.so
    echo "== $L round $r" >> gpurun_out/r04e_mmq_ab.log
    MI355X_LIB=$lib timeout -k 10 150 python tools/prefill_bench.py >> gpurun_out/r04e_mmq_ab.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/r04e_mmq_ab.log | sed 's/total.*gemm/gemm/'
TAG=r04 bash tools/prof_prefill.sh || exit $?
