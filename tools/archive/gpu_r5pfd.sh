#!/bin/bash
# Round 5: B = 1 decode with the finished gate|up workgroups reading the down projection's first round of rows
# into the caches (gemv_body.h PGMI_GU_PFD, probe builds: 1 = 8 MB, 2 = 16 MB) -- same-box A/B.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5pfd
mkdir -p $OUT
timeout -k 10 1000 bash $R/tools/ab_variants.sh "pfd1 pfd2" 3 b1 $OUT/ab_b1.txt
echo done
