#!/bin/bash
# Round 5: what the graph-replayed decode token costs with its launches emptied, without a
# profiler in the way. bench.py's headline token (hipGraph replay) on the product library,
# then on the diagnostic build (libfdiag: KQ_ROWS_DIAG, KQ_GEMV_DIAG, KQ_ATTN_DIAG) with
# the attention launches empty (ATTN_DIAG=4), the GEMVs empty (GEMV_DIAG=256), and both:
# the last is the launch chain's floor (every launch kept, each returning at entry).
#   build: make -C ggml-neon-opt_amd variant NAME=fdiag VFLAGS="-DKQ_ROWS_DIAG=1 -DKQ_GEMV_DIAG=1 -DKQ_ATTN_DIAG=1"
#          plus kq_ops.hip with the same flags (tools/token_floor.sh's header in DESIGN §7)
# LIST="tag lib knob=v ..." lines replace the default variants (e.g. the attention's
# diagnostic stops: ATTN_DIAG=5 q/k/v + rope only, 1 + the cache loads, 2 + KQ, 3 + soft_max).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
FLAGS="--steps 128 --warmup 16 --no-cpu-baseline --no-large --no-prefill --no-chain --no-8b --no-70b --no-collectives --tg 0"
D=ggml-neon-opt_amd/lib/variants/libfdiag.so
P=ggml-neon-opt_amd/lib/libggml_mi355x.so
for model in ${MODELS:-tinyllama-1.1b llama-3-8b}; do
  for r in 1 2; do
    while read -r tag lib knobs; do
      kargs=""
      for k in $knobs; do [ "$k" = "-" ] || kargs="$kargs --knob $k"; done
      MI355X_LIB=$lib timeout -k 10 300 python -u bench.py --model $model $FLAGS $kargs > gpurun_out/tf_tmp.json 2> gpurun_out/tf_tmp.err
      rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $tag"; tail -5 gpurun_out/tf_tmp.err; exit $rc; }
      tail -1 gpurun_out/tf_tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$model', '$r', '$tag', d['value'], d['ms_per_step'], d['config']['stages_per_token'])"
    done <<LIST
${LIST:-product $P -
diag $D -
attn_empty $D ATTN_DIAG=4
gemv_empty $D GEMV_DIAG=256
all_empty $D GEMV_DIAG=256 ATTN_DIAG=4}
LIST
  done
done
