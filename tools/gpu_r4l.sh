#!/bin/bash
# HIP runtime placement of kernel arguments: the TinyLlama / Llama-3-8B tokens with
# HIP_FORCE_DEV_KERNARG=1 (kernargs in device memory) and =0 against the default, interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/r04l_kernarg.log
for r in 1 2; do
  for kv in default 1 0; do
    for model in tinyllama-1.1b llama-3-8b; do
      if [ $kv = default ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$kv; fi
      timeout -k 10 200 python bench.py --model $model --steps 64 --warmup 8 --no-cpu-baseline --no-large --no-prefill \
          --no-8b --no-70b --no-chain --tg 0 --no-collectives > gpurun_out/kv.json 2>&1 || exit $?
      echo "kernarg=$kv $model $(grep -o '"value": [0-9.]*' gpurun_out/kv.json | head -1)" | tee -a gpurun_out/r04l_kernarg.log
    done
  done
done
unset HIP_FORCE_DEV_KERNARG
