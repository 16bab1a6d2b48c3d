#!/bin/bash
# Round 5: M = 288 Gemma down / o_proj GEMMs on row tilings that divide 288 (P96x64 rings: cfg 28 s4, 29 s3) over
# K splits, beside the current plans (tools/gemm_sweep.py, in isolation, hot and cold).
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5y
mkdir -p $OUT
for mode in "" "--cold"; do
  timeout -k 10 300 python3 -u $R/tools/gemm_sweep.py t_down --cfgs 28,29,34,31,30 --splits 1,2,3,4,6,8 --all $mode \
      >> $OUT/sweep_down$mode.txt 2>&1
  timeout -k 10 300 python3 -u $R/tools/gemm_sweep.py t_o --cfgs 28,29,34,31 --splits 1,2,3,4 --all $mode \
      >> $OUT/sweep_o$mode.txt 2>&1
done
echo done
