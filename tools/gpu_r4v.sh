#!/bin/bash
# Final round-4 measurement: smoke, the default bench line, then the TinyLlama token profile
# (kernel trace + FETCH / WRITE passes) summarised on the box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/profiles_out
timeout -k 10 120 python -c "import __graft_entry__ as e; e.smoke()" > gpurun_out/r04v_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r04v_smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/r04v_bench.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' gpurun_out/r04v_bench.log | head -1
TAG=r04v timeout -k 10 600 bash tools/profile_token.sh > /dev/null || exit $?
python3 tools/prof_summary.py gpurun_out/prof_r04v profiles/r04v_token --warmup 8 --steps 64 --launches 112 --pmc-warmup 2 \
    --pmc-steps 16 --bench-json gpurun_out/prof_r04v/bench_trace.log --kinds gpurun_out/prof_r04v/kinds.json > /dev/null || exit $?
cp profiles/r04v_token_summary.* gpurun_out/profiles_out/
cp gpurun_out/prof_r04v/trace/run_kernel_stats.csv gpurun_out/profiles_out/r04v_kernel_stats.csv
rm -f gpurun_out/prof_r04v/trace/run_kernel_trace.csv
head -30 profiles/r04v_token_summary.md
