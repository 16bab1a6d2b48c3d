#!/bin/bash
# Round 5: in-situ plan sweep (whole generate-loop LM prefill timed per candidate) of the M = 288 o_proj and down
# on the P96x64 rings (cfg 28 / 29: row tiles that divide 288) beside the current plans.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5z
mkdir -p $OUT
timeout -k 10 600 python3 -u $R/tools/probes/plan_sweep.py --target lm --shapes o,down --cfgs 28,29,34,31,30 \
    --splits 1,2,3,4,6,8 --iters 20 --rel-tol 5e-2 > $OUT/lm_sweep.txt 2>&1
echo done
