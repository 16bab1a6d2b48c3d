#!/bin/bash
# Round 5: B = 1 gate|up and down GEMVs with two rows (row pairs) per wave (probe builds PGMI_GU_RPW2 / PGMI_DN_RPW2,
# grid caps 512 / 1,024 and 256 / 512): the B = 1 model tests on gr1024 and dr256, then same-box B = 1 A/B.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5rpw
mkdir -p $OUT
P=$R/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi
for v in gr1024 dr256; do
  PGMI_LIB_PATH=$P/libpgmi_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
      $R/tests/test_gpu_full.py > $OUT/tests_$v.log 2>&1
done
echo tests done
timeout -k 10 900 bash $R/tools/ab_variants.sh "gr512 gr1024 dr256 dr512" 2 b1 $OUT/ab_b1.txt
echo done
