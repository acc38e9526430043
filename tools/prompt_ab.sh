#!/bin/bash
# A/B of prompt attention builds: LIBS="name=path ..." (default: the product library against
# lib/variants/libpold.so), TinyLlama pp512 eager per-kernel sums, interleaved ROUNDS times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIBS=${LIBS:-"new=ggml-neon-opt_amd/lib/libggml_mi355x.so old=ggml-neon-opt_amd/lib/variants/libpold.so"}
for r in $(seq ${ROUNDS:-2}); do
    for kv in $LIBS; do
        echo "== ${kv%%=*}"
        MI355X_LIB=${kv#*=} timeout -k 10 120 python3 tools/prompt_profile.py ${MODEL:-tinyllama-1.1b} 2>/dev/null | grep -E "${GREP:-attn_prompt|kv_store|total}" || exit 1
    done
done
