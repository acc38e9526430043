#!/bin/bash
# Builds the committed HEAD (or REV) library as lib/variants/lib${NAME:-pold}.so: the baseline
# of an A/B against the working tree (tools/prompt_ab.sh, tools/mmq_libs.sh).
set -eu
cd "$(dirname "$0")/.."
D=ggml-neon-opt_amd/build/head
rm -rf $D && mkdir -p $D
git archive ${REV:-HEAD} ggml-neon-opt_amd include | tar -x -C $D
make -s -C $D/ggml-neon-opt_amd -j8
mkdir -p ggml-neon-opt_amd/lib/variants
cp $D/ggml-neon-opt_amd/lib/libggml_mi355x.so ggml-neon-opt_amd/lib/variants/lib${NAME:-pold}.so
rm -rf $D
