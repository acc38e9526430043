#!/bin/bash
# Where the decode GEMVs' vector instructions go: the wave-state PMC pass on the diagnostic
# build (lib/variants/libdiag.so) with each piece switched off (MI355X_GEMV_DIAG bits: 8 no dot
# products / records, 64 no quantization, 32 no norm / swiglu transform, 128 no swiglu epilogue).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MI355X_LIB=$PWD/ggml-neon-opt_amd/lib/variants/libdiag.so
for d in 0 8 64 32 128; do
  echo "== GEMV_DIAG=$d"
  TAG=d$d KNOBS="--knob GEMV_DIAG=$d" bash tools/prof_decode_pmc.sh | grep kq_rows || exit $?
done
