#!/bin/bash
# Round 5: B = 1 decode with the attention launch's idle CUs reading the layer's o_proj rows (pf1) and also the
# first gate|up row groups (pf3) into the caches (kernels_attn.hip PGMI_DEC_PF, probe builds) -- same-box A/B.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5pf
mkdir -p $OUT
timeout -k 10 1000 bash $R/tools/ab_variants.sh "pf1 pf3" 3 b1 $OUT/ab_b1.txt
echo done
