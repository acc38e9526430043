#!/bin/bash
# Round 5: attention batching on/off (product vs anob): decode tokens of both models + tg1024/tg20.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/ab_libs.sh default anob > gpurun_out/r5t_ab_libs.txt 2>&1 || { tail -5 gpurun_out/r5t_ab_libs.txt; exit 1; }
grep -E "^(default|anob) " gpurun_out/r5t_ab_libs.txt | python3 -c "
import sys,ast
for l in sys.stdin:
    p=l.split(' ',4); d=ast.literal_eval(p[4].strip())
    print(p[0], p[1], p[2], {k:v for k,v in d.items() if 'attn' in k})"
LIBS="lib/libggml_mi355x.so lib/variants/libanob.so" bash tools/attn_tg_ab.sh > gpurun_out/r5t_attn_ab.txt 2>&1
cat gpurun_out/r5t_attn_ab.txt
