#!/bin/bash
# Round 5: the one-pass key-split prefill attention at forced key-range counts (1 / 2 / 4 / auto) on the Gemma
# 224 / 448 and SigLIP 448 shapes (tools/probes/attn_bench.py).
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5x
mkdir -p $OUT
ATTN_SHAPES=gemma224,gemma448,siglip448 timeout -k 10 300 python3 -u $R/tools/probes/attn_bench.py -1 9 91 92 94 > $OUT/attn.txt 2>&1
echo done
