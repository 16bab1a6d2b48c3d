#!/bin/bash
# Round 6: what paces the M = 288 MLP GEMMs -- the same cold isolated sweep on the diagnostic builds
# (tools/build_variant.sh: PGMI_GEMM_DIAG=1 compute waves issue no MFMA, =2 no LDS-DMA is issued)
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6d
mkdir -p $OUT
cd $R
P=$R/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi
for v in diag1 diag2; do
  PGMI_LIB_PATH=$P/libpgmi_$v.so timeout -k 10 300 python -u tools/gemm_sweep.py t_gateup t_down t448_gateup --cold --all \
      --cfgs 30,31,34,37,40 --splits 1,8,12 > $OUT/iso_$v.txt 2>&1
  echo $v done
done
