#!/bin/bash
# Round 5: after the 8-wave gate|up / down: q|k|v and o_proj with 16 K-split waves (probe builds PGMI_QKV_W16 /
# PGMI_O_W16) and the down projection on 64 x 8 workgroups (PGMI_DN_WG=64): the batch tests on q16 and o16, then
# same-box B = 8 A/B.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5w16
mkdir -p $OUT
P=$R/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi
for v in q16 o16; do
  PGMI_LIB_PATH=$P/libpgmi_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
      $R/tests/test_gpu_full_batch.py > $OUT/tests_$v.log 2>&1
done
echo tests done
timeout -k 10 900 bash $R/tools/ab_variants.sh "dw64 q16 o16" 3 b8 $OUT/ab_b8.txt
echo done
