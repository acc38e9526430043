#!/bin/bash
# rocprofv3 kernel trace + stats of the default bench, then a separate PMC pass
# (FETCH_SIZE) of the same command. Outputs under gpurun_out/prof_<tag>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
ARGS=${BENCH_ARGS:-"--steps 64 --warmup 8 --no-cpu-baseline --no-large"}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_trace.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_pmc_fetch.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_pmc_write.log" 2>&1 || exit $?
find "$OUT" -name "*.csv" | head -50
