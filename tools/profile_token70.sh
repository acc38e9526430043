#!/bin/bash
# Round 6: rocprofv3 token profile (kernel trace + FETCH_SIZE / WRITE_SIZE passes) of the Llama-3-70B token on one GPU.
set -u
cd "${GRAFT_REPO_ROOT}"
TAG=r06f70 BENCH_ARGS="--model llama-3-70b --steps 12 --warmup 2 --no-cpu-baseline --no-large --no-prefill --no-chain --no-8b --no-70b --tg 0" \
  PMC_ARGS="--model llama-3-70b --steps 3 --warmup 1 --no-graph --no-cpu-baseline --no-large --no-prefill --no-chain --no-8b --no-70b --tg 0" \
  timeout -k 10 700 bash tools/profile_token.sh > gpurun_out/prof_r06f70.log 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/prof_r06f70.log; exit 1; }
O=gpurun_out/prof_r06f70
grep "^{" $O/bench_trace.log | tail -1 > $O/bench.json
python3 tools/prof_summary.py $O gpurun_out/r06f70_token_summary --warmup 2 --steps 12 --launches 402 --pmc-warmup 1 --pmc-steps 3 \
    --bench-json $O/bench.json --kinds $O/kinds.json > $O/summary.log 2>&1 || { echo summary failed; tail -5 $O/summary.log; }
find $O -name "*.csv" -size +1M -delete
head -40 gpurun_out/r06f70_token_summary.md
