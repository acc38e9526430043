#!/bin/bash
# Prompt attention ablations (timing only): KQ_PROMPT_DIAG builds of kq_ops
# (make variant-ops NAME=pd<v> VFLAGS=-DKQ_PROMPT_DIAG=<v>), TinyLlama pp512 eager per-kernel sums.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
    for v in base 1 2 4 7; do
        if [ $v = base ]; then lib=ggml-neon-opt_amd/lib/libggml_mi355x.so; else lib=ggml-neon-opt_amd/lib/variants/libpd$v.so; fi
        echo "== $v"
        MI355X_LIB=$lib timeout -k 10 120 python3 tools/prompt_profile.py ${MODEL:-tinyllama-1.1b} 2>/dev/null | grep -E "attn_prompt|total" || exit 1
    done
done
