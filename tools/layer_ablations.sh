#!/bin/bash
# Round 5: persistent-layer ablations (stamps builds): product, no dots, no DMA, neither.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in lst ld1 ld2 ld3; do
  MI355X_LIB=ggml-neon-opt_amd/lib/variants/lib$v.so timeout -k 10 200 python -u tools/layer_stamps.py --model llama-3-8b --tokens 4 > gpurun_out/${TAG:-r5d}_$v.log 2>&1
  rc=$?; echo "== $v rc=$rc"; tail -18 gpurun_out/${TAG:-r5d}_$v.log | awk '{print $1, $2, $3}' | tr '\n' ' '; echo
  [ $rc -eq 0 ] || exit $rc
done
