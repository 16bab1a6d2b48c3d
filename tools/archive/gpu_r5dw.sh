#!/bin/bash
# Round 5: the batched down projection with 8 K-split waves (KW 256) per K slice on 32 / 16 x 8 workgroups (probe
# builds PGMI_DN_W8): the batch tests on dw32, then same-box B = 8 A/B against 4 waves x 512 on 32 x 8.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5dw
mkdir -p $OUT
PGMI_LIB_PATH=$R/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi/libpgmi_dw32.so timeout -k 10 600 \
    python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $R/tests/test_gpu_full_batch.py > $OUT/tests.log 2>&1
echo tests done
timeout -k 10 900 bash $R/tools/ab_variants.sh "dw32 dw16" 3 b8 $OUT/ab_b8.txt
echo done
