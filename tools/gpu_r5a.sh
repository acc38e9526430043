#!/bin/bash
# Round 5: persistent decode layer -- parity tests first, then the engine A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_layer.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r5a_layer_tests.log 2>&1
rc=$?; echo "layer tests rc=$rc"; tail -25 gpurun_out/r5a_layer_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/layer_ab.py --rounds 3 --steps 64 --layer-profile > gpurun_out/r5a_layer_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r5a_layer_ab.log | cut -c1-1500
exit $rc
