#!/bin/bash
# Round 6: the in-wave reload mode of k_gemm_w (cfgs 51-53: R144q, R288w, R128q) against W288n on the
# M = 288 MLP GEMMs (and the 448 px gate|up), cold isolated and in situ
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6i
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u tools/gemm_sweep.py t_gateup t_down t448_gateup --cold --all --iters 40 --cfgs 31,37,51,52,53 \
    --splits 1,8,16 > $OUT/iso.txt 2>&1
echo iso done
timeout -k 10 400 python -u tools/probes/plan_sweep.py --target lm --shapes gateup,down --cfgs 31,51,52,53 \
    --splits 8,16 --rel-tol 5e-2 > $OUT/insitu.txt 2>&1
echo insitu done
