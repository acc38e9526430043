#!/bin/bash
# Decode-token A/B of library builds: the decode parity tests on the first candidate, then
# the TinyLlama and Llama-3-8B tokens for every library, interleaved twice.
#   usage (GPU box): bash tools/ab_libs.sh NAME... (lib/variants/libNAME.so; "default": the product)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$PWD/ggml-neon-opt_amd/lib/variants
first=""
for L in "$@"; do [ "$L" != default ] && [ -z "$first" ] && first=$L; done
if [ -n "$first" ]; then
  MI355X_LIB=$V/lib$first.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py -x -q \
      --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_libs_tests.log 2>&1
  rc=$?; echo "tests on $first:"; tail -2 gpurun_out/ab_libs_tests.log; [ $rc -eq 0 ] || exit $rc
fi
OUT=gpurun_out/ab_libs.log
: > $OUT
for r in 1 2; do
  for L in "$@"; do
    for model in tinyllama-1.1b llama-3-8b; do
      if [ $L = default ]; then unset MI355X_LIB; else export MI355X_LIB=$V/lib$L.so; fi
      timeout -k 10 200 python bench.py --model $model --steps 64 --warmup 8 --no-cpu-baseline --no-large \
          --no-prefill --no-8b --no-70b --no-chain --tg 0 --no-collectives > gpurun_out/ab_one.json 2>/dev/null || exit $?
      python - "$L $model" >> $OUT <<'PY' || exit $?
import json, sys
d = json.loads(open("gpurun_out/ab_one.json").read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], d["ms_per_step"], {k.replace("kq::", ""): v["us_per_launch"] for k, v in d["kernels"].items()}, flush=True)
PY
    done
  done
done
unset MI355X_LIB
cat $OUT
