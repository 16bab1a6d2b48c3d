#!/bin/bash
# Round 6: the M = 288 (224 px) Gemma MLP GEMMs on the W144 tiles (one 144-row wave row, no padded rows) --
# cold isolated sweep (tools/gemm_sweep.py) and in situ (whole LM prefill per candidate, plan_sweep.py)
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6b
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u tools/gemm_sweep.py t_gateup --cold --all --cfgs 30,31,38,39,40 --splits 1 > $OUT/iso_gateup.txt 2>&1
echo iso gateup done
timeout -k 10 300 python -u tools/gemm_sweep.py t_down --cold --all --cfgs 30,34,38,39,40 --splits 4,8,12,16 > $OUT/iso_down.txt 2>&1
echo iso down done
timeout -k 10 400 python -u tools/probes/plan_sweep.py --target lm --shapes gateup,down --cfgs 31,34,38,39,40 \
    --splits 4,8,16 --rel-tol 5e-2 > $OUT/insitu.txt 2>&1
echo insitu done
