#!/bin/bash
# Round 6: what paces k_gemm_w / k_gemm_wp (ping-pong) / k_gemm_h (32-deep ring) on the M = 288 gate|up and
# down: the same cold isolated sweep on the product build and on the diagnostic builds (PGMI_GEMM_DIAG=1: no
# MFMA, =2: no LDS-DMA, =3: neither -- the barrier / fragment-read / epilogue skeleton)
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6f
mkdir -p $OUT
cd $R
P=$R/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi
for v in prod diag1 diag2 diag3; do
  if [ $v = prod ]; then unset PGMI_LIB_PATH; else export PGMI_LIB_PATH=$P/libpgmi_$v.so; fi
  timeout -k 10 300 python -u tools/gemm_sweep.py t_gateup t_down --cold --all --iters 40 \
      --cfgs 31,41,45 --splits 1,8 > $OUT/iso_$v.txt 2>&1
  echo $v done
done
