#!/bin/bash
# Round 5: the batched gate|up and down grids re-swept after the peeled loop (probe builds PGMI_GU_WG / PGMI_DN_WG):
# same-box B = 8 A/B against the default 256 / 32 x 8 workgroups.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5grid
mkdir -p $OUT
timeout -k 10 1000 bash $R/tools/ab_variants.sh "gu512 gu128 dn64 dn16" 2 b8 $OUT/ab_b8.txt
echo done
