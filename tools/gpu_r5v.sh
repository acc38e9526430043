#!/bin/bash
# Round 5: the 12-wave 192-row prefill tile (MI355X_MMQ_TILE192): parity, then GEMM timings against AUTO.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ops.py -k "mmq" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5v_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5v_tests.log; [ $rc -eq 0 ] || exit $rc
RUNS="tile128: tile192: auto: tile128: tile192:" PREFILL_TYPES=12 bash tools/mmq_libs.sh > gpurun_out/r5v_mmq12.txt 2>&1; grep -v amdgpu gpurun_out/r5v_mmq12.txt | sed 's/kq::kq_quantize.*//'
RUNS="tile128: tile192: auto:" PREFILL_TYPES=13 bash tools/mmq_libs.sh > gpurun_out/r5v_mmq13.txt 2>&1; grep -v amdgpu gpurun_out/r5v_mmq13.txt | sed 's/kq::kq_quantize.*//'
