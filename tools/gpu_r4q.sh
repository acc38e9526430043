#!/bin/bash
# Llama-3-8B decode token under rocprofv3 (kernel trace + FETCH / WRITE passes), summarised on
# the box (tools/prof_summary.py), raw kernel trace dropped (gpurun_out is capped at 64 MiB).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/profiles_out
export BENCH_ARGS="--model llama-3-8b --steps 32 --warmup 4 --no-cpu-baseline --no-large --no-prefill --no-chain --no-8b --no-70b --tg 0 --no-collectives"
export PMC_ARGS="--model llama-3-8b --steps 8 --warmup 2 --no-graph --no-cpu-baseline --no-large --no-prefill --no-chain --no-8b --no-70b --tg 0 --no-collectives"
TAG=r04q timeout -k 10 900 bash tools/profile_token.sh > /dev/null || exit $?
python3 tools/prof_summary.py gpurun_out/prof_r04q profiles/r04q_token8b --warmup 4 --steps 32 --launches 162 --pmc-warmup 2 \
    --pmc-steps 8 --bench-json gpurun_out/prof_r04q/bench_trace.log --kinds gpurun_out/prof_r04q/kinds.json > /dev/null || exit $?
cp profiles/r04q_token8b_summary.* gpurun_out/profiles_out/
rm -f gpurun_out/prof_r04q/trace/run_kernel_trace.csv
head -30 profiles/r04q_token8b_summary.md
