#!/bin/bash
# kq_mmf A/B of run-time knobs (env), interleaved on one box: tools/mmf_ab.sh "ENV1" "ENV2" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for pass in 1 2; do
  for cfg in "$@"; do
    echo "== pass $pass: $cfg"
    env MI355X_PREFILL=${PREC:-f16_all} $cfg timeout -k 10 120 python -u tools/prefill_bench.py 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
