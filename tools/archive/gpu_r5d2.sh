#!/bin/bash
# Round 5: the batched gate|up with 8 K-split waves, one-deep (w8a) or two-deep register streams (d2a: 256
# workgroups, d2b: 128) after the peeled loop (probe builds PGMI_GU_W8 / PGMI_GU_D2): the batch tests on d2a, then
# same-box B = 8 A/B against 4 waves x 256 workgroups.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5d2
mkdir -p $OUT
PGMI_LIB_PATH=$R/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi/libpgmi_d2a.so timeout -k 10 600 \
    python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $R/tests/test_gpu_full_batch.py > $OUT/tests.log 2>&1
echo tests done
timeout -k 10 900 bash $R/tools/ab_variants.sh "w8a d2a d2b" 3 b8 $OUT/ab_b8.txt
echo done
