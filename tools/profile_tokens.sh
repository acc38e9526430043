#!/bin/bash
# Round 5: rocprofv3 token profiles (kernel trace + stats; FETCH_SIZE / WRITE_SIZE PMC passes)
# of the default TinyLlama token and the Llama-3-8B token.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TT=${TAG_TINY:-r05v}; T8=${TAG_8B:-r05q}
TAG=$TT timeout -k 10 500 bash tools/profile_token.sh > gpurun_out/prof_$TT.log 2>&1 || { echo "tiny rc=$?"; tail -5 gpurun_out/prof_$TT.log; exit 1; }
echo tiny ok
TAG=$T8 BENCH_ARGS="--model llama-3-8b --steps 32 --warmup 4 --no-cpu-baseline --no-large --no-prefill --no-chain --no-8b --no-70b --tg 0" \
  PMC_ARGS="--model llama-3-8b --steps 8 --warmup 2 --no-graph --no-cpu-baseline --no-large --no-prefill --no-chain --no-8b --no-70b --tg 0" \
  timeout -k 10 500 bash tools/profile_token.sh > gpurun_out/prof_$T8.log 2>&1 || { echo "8b rc=$?"; tail -5 gpurun_out/prof_$T8.log; exit 1; }
echo 8b ok
# summaries on the box (the raw traces stay there: too large to copy back)
for t in $TT:112 $T8:162; do
  tag=${t%%:*}; n=${t##*:}; O=gpurun_out/prof_$tag
  if [ $tag = $TT ]; then W=8; S=64; PW=2; PS=16; else W=4; S=32; PW=2; PS=8; fi
  grep "^{" $O/bench_trace.log | tail -1 > $O/bench.json
  python3 tools/prof_summary.py $O gpurun_out/${tag}_token --warmup $W --steps $S --launches $n --pmc-warmup $PW --pmc-steps $PS \
    --bench-json $O/bench.json --kinds $O/kinds.json > $O/summary.log 2>&1 || { echo "summary $tag failed"; tail -5 $O/summary.log; }
  find $O -name "*.csv" -size +1M -delete
done
ls gpurun_out/*_token_summary.* 
