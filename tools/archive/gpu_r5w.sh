#!/bin/bash
# Round 5: the batched gate|up grid over its fragment-major image: 256 / 384 workgroups against 512 (default), B = 8.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5w
mkdir -p $OUT
timeout -k 10 900 bash $R/tools/ab_variants.sh "gu256 gu384" 4 b8 $OUT/ab_b8.txt
echo done
