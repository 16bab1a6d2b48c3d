#!/bin/bash
# Round 5: what paces the M = 288 / 256 prefill GEMMs -- each shape hot (same weights every call: L2 / MALL)
# and cold (rotating weight copies: HBM), over tile plans and K splits.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5b
mkdir -p $OUT
for mode in "" "--cold"; do
  timeout -k 10 300 python3 -u $R/tools/gemm_sweep.py t_down --cfgs 30,31,34,23,20,6 --splits 1,2,4,8,16 --all $mode \
      >> $OUT/sweep_down$mode.txt 2>&1
  timeout -k 10 300 python3 -u $R/tools/gemm_sweep.py t_gateup --cfgs 30,31,34,23,20,6,36,37 --splits 1 --all $mode \
      >> $OUT/sweep_gateup$mode.txt 2>&1
  timeout -k 10 300 python3 -u $R/tools/gemm_sweep.py v_fc2 v_fc1 v_qkv v_out --cfgs 25,28,24,26,14,15,16,17,32,34,35 \
      --splits 1,2,3,4 --all $mode >> $OUT/sweep_vision$mode.txt 2>&1
done
echo done
