#!/bin/bash
# Launch-slot cost (tools/slot_cost.hip), the attention stops, then the token profile with its
# summary made on the box (the raw kernel trace stays there: gpurun_out is capped at 64 MiB).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 tools/_build/slot_cost > gpurun_out/slot_cost.log 2>&1 || exit $?
cat gpurun_out/slot_cost.log
timeout -k 10 900 bash tools/attn_stops.sh || exit $?
TAG=r04h timeout -k 10 600 bash tools/profile_token.sh > /dev/null || exit $?
python3 tools/prof_summary.py gpurun_out/prof_r04h profiles/r04h_token --warmup 8 --steps 64 --launches 112 --pmc-warmup 2 \
    --pmc-steps 16 --bench-json gpurun_out/prof_r04h/bench_trace.log --kinds gpurun_out/prof_r04h/kinds.json > /dev/null || exit $?
mkdir -p gpurun_out/profiles_out && cp profiles/r04h_token_summary.* gpurun_out/profiles_out/
rm -f gpurun_out/prof_r04h/trace/run_kernel_trace.csv
head -12 profiles/r04h_token_summary.md
