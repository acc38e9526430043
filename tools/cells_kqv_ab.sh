#!/bin/bash
# Round 6: kq_attn_cells_kqv forms — per-kernel times of the probe on the product (16 threads per
# output chain), cold (4 per output, round-6 first form), cstop1 / cstop2 (B stops after its
# loads / soft_max), then the tg A/B of tools/cells_ab.sh on LIBS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=gpurun_out/cells_kqv_probe.txt
: > $P
for l in ${PLIBS:-lib/libggml_mi355x.so}; do
  echo "== $l" >> $P
  MI355X_LIB=ggml-neon-opt_amd/$l timeout -k 10 200 python -u tools/attn_cells_probe.py > gpurun_out/probe_tmp.txt 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/probe_tmp.txt >> $P; [ $rc -eq 0 ] || { cat $P; exit $rc; }
done
cat $P
