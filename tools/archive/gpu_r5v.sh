#!/bin/bash
# Round 5: grid sizes of the batched gate|up (512 default; 1,024 / 256) and down (32 x 8 default; 64 / 16 x 8) GEMVs
# over their fragment-major images, same box, B = 8 (probe builds libpgmi_{dn64,dn16,gu1024,gu256}.so).
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5v
mkdir -p $OUT
timeout -k 10 900 bash $R/tools/ab_variants.sh "dn64 dn16 gu1024 gu256" 2 b8 $OUT/ab_b8.txt
echo done
