#!/bin/bash
# Round 5: persistent decode layer -- parity tests, phase stamps, engine A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r5c}
timeout -k 10 400 python -u -m pytest tests/test_gpu_layer.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_layer_tests.log 2>&1
rc=$?; echo "layer tests rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/${T}_layer_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/layer_stamps.py --model llama-3-8b > gpurun_out/${T}_stamps8b.log 2>&1
rc=$?; echo "stamps rc=$rc"; tail -19 gpurun_out/${T}_stamps8b.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/layer_ab.py --rounds 3 --steps 64 > gpurun_out/${T}_layer_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; cat gpurun_out/${T}_layer_ab.log | grep model | cut -c1-400
exit $rc
