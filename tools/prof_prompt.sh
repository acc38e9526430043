#!/bin/bash
# rocprofv3 kernel trace + stats of one graph-replayed pp512 prompt (TinyLlama, then
# Llama-3-8B) through LlamaDecoder.prompt (tools/prompt_profile.py runs it eagerly with
# the launch-timing hook; this is the graph-replayed trace of the bench's pp512 figure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02}
OUT=gpurun_out/prof_prompt_$TAG
mkdir -p "$OUT"
for m in tinyllama-1.1b llama-3-8b; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$m" -o run -- \
        python3 tools/prompt_graph_run.py "$m" > "$OUT/$m.log" 2>&1 || exit $?
done
find "$OUT" -name "*stats.csv"
