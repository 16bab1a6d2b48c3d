#!/bin/bash
# Round 5: the decode attention's V rows loaded after its K / mask / q fragments (probe build PGMI_ATT_VLAST), so the
# score MFMAs wait for K and q only: the B = 1 and batch tests on the variant, then same-box A/Bs at B = 1 and 8.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5vl
mkdir -p $OUT
PGMI_LIB_PATH=$R/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi/libpgmi_vl.so timeout -k 10 600 \
    python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $R/tests/test_gpu_full.py \
    $R/tests/test_gpu_full_batch.py > $OUT/tests.log 2>&1
echo tests done
timeout -k 10 600 bash $R/tools/ab_variants.sh "vl" 3 b1 $OUT/ab_b1.txt
timeout -k 10 600 bash $R/tools/ab_variants.sh "vl" 3 b8 $OUT/ab_b8.txt
echo done
