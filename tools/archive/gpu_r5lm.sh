#!/bin/bash
# Round 5: the batched lm_head on the register-streamed MFMA GEMV (peeled loop, row-major tied embedding, 4 waves
# splitting K, rows staged + final-normed per workgroup) on 512 / 1,024 / 2,048 workgroups (probe builds
# PGMI_LM_MF) against the LDS-DMA ring: the batch tests on lm1024, then same-box B = 8 A/B.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5lm
mkdir -p $OUT
P=$R/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi
PGMI_LIB_PATH=$P/libpgmi_lm1024.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    $R/tests/test_gpu_full_batch.py > $OUT/tests.log 2>&1
echo tests done
timeout -k 10 900 bash $R/tools/ab_variants.sh "lm512 lm1024 lm2048" 3 b8 $OUT/ab_b8.txt
echo done
