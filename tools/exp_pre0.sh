#!/bin/bash
# Ring issued before the activation wait (KQ_ROWS_PRE0=3, lib/variants/libp3.so) against the
# product (one step): per-wave stamps of both (diag builds), the large GEMVs, and the
# TinyLlama / Llama-3-8B tokens interleaved. Build first (CPU):
#   make -C ggml-neon-opt_amd variant NAME=p3 VFLAGS="-DKQ_ROWS_PRE0=3"
#   make -C ggml-neon-opt_amd variant NAME=diag VFLAGS="-DKQ_ROWS_DIAG=1 -DKQ_GEMV_DIAG=1"
#   make -C ggml-neon-opt_amd variant NAME=diagp3 VFLAGS="-DKQ_ROWS_DIAG=1 -DKQ_GEMV_DIAG=1 -DKQ_ROWS_PRE0=3"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=ggml-neon-opt_amd/lib/variants
for L in diag diagp3; do
  echo "== stamps $L"
  MI355X_LIB=$PWD/$V/lib$L.so timeout -k 10 150 python -u tools/stamps.py rows 2>&1 | grep -v amdgpu.ids || exit $?
done
for r in 1 2; do
  for L in default p3; do
    echo "== large $L"
    if [ $L = default ]; then unset MI355X_LIB; else export MI355X_LIB=$PWD/$V/lib$L.so; fi
    timeout -k 10 150 python -u tools/gemv_large_ab.py 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
unset MI355X_LIB
timeout -k 10 400 bash tools/ab_token.sh default $V/libp3.so || exit $?
BENCH_ARGS="--model llama-3-8b" timeout -k 10 400 bash tools/ab_token.sh default $V/libp3.so || exit $?
