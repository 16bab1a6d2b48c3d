#!/bin/bash
# Round 6: plan re-sweeps of the large-M Gemma MLP GEMMs with the round's new tiles, in situ: 8 images
# (M = 2304: E192 = 12 row tiles, 6 rounds of 256, against E256's 9 tiles = 4.5 rounds) and 448 px (M = 1056)
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6g
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u tools/probes/plan_sweep.py --target lm --batch 8 --shapes gateup,down --cfgs 36,37,30,41,46 \
    --splits 1,2,3 --iters 10 --rel-tol 5e-2 > $OUT/insitu_b8.txt 2>&1
echo b8 done
timeout -k 10 500 python -u tools/probes/plan_sweep.py --target lm --px 448 --shapes gateup,down --cfgs 36,37,41,46 \
    --splits 4,5,8 --iters 10 --rel-tol 5e-2 > $OUT/insitu_448.txt 2>&1
echo 448 done
timeout -k 10 300 python -u tools/probes/plan_sweep.py --target lm --shapes attn --iters 20 > $OUT/insitu_attn224.txt 2>&1
echo attn done
