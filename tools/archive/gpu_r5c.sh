#!/bin/bash
# Round 5: where the prefill GEMMs' k-loop time goes -- each in-use plan timed with the product build, a build
# whose compute waves issue no MFMA (fragments still read, -DPGMI_GEMM_DIAG=1) and a build whose LDS-DMA stages
# load nothing (-DPGMI_GEMM_DIAG=2); tools/build_variant.sh builds them in-tree before the call.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5c
mkdir -p $OUT
P=$R/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi
for lib in libpgmi libpgmi_diag1 libpgmi_diag2; do
  echo "== $lib" >> $OUT/diag.txt
  PGMI_LIB_PATH=$P/$lib.so timeout -k 10 200 python3 -u $R/tools/gemm_sweep.py t_gateup --cfgs 31,37,20 --splits 1 --all >> $OUT/diag.txt 2>&1
  PGMI_LIB_PATH=$P/$lib.so timeout -k 10 200 python3 -u $R/tools/gemm_sweep.py t_down --cfgs 34,31,30 --splits 4,8,16 --all >> $OUT/diag.txt 2>&1
  PGMI_LIB_PATH=$P/$lib.so timeout -k 10 200 python3 -u $R/tools/gemm_sweep.py t448_gateup t448_down --cfgs 37 --splits 1,5 --all >> $OUT/diag.txt 2>&1
  PGMI_LIB_PATH=$P/$lib.so timeout -k 10 200 python3 -u $R/tools/gemm_sweep.py v_fc1 v_fc2 v_qkv v_out --cfgs 25,28 --splits 1,3,4 --all >> $OUT/diag.txt 2>&1
done
echo done
