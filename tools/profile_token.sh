#!/bin/bash
# rocprofv3 kernel trace + stats of the bench command, then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) of a shorter eager run of the same workload (counter
# collection serializes every dispatch; per-launch bytes do not depend on graph
# replay). Outputs under gpurun_out/prof_<tag>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
ARGS=${BENCH_ARGS:-"--steps 64 --warmup 8 --no-cpu-baseline --no-large --no-prefill --no-chain --no-8b --no-70b --tg 0"}
PMC_ARGS=${PMC_ARGS:-"--steps 16 --warmup 2 --no-graph --no-cpu-baseline --no-large --no-prefill --no-chain --no-8b --no-70b --tg 0"}
BENCH_KINDS_OUT="$OUT/kinds.json" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_trace.log" 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 bench.py $PMC_ARGS > "$OUT/bench_pmc_fetch.log" 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 bench.py $PMC_ARGS > "$OUT/bench_pmc_write.log" 2>&1 || exit $?
find "$OUT" -name "*.csv"
