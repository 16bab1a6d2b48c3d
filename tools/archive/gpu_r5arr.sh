#!/bin/bash
# Round 5: the decode GEMVs' reduction and stream schedule (probe builds): ARRIVE (kernels_gemv_mfma.hip /
# gemv_body.h PGMI_MF_ARRIVE: the K-split waves of a group meet through an LDS arrival count instead of two
# barriers), PEEL (PGMI_MF_PEEL: the batched GEMVs' last group peeled, so the next group's stream issue is
# unconditional and each MFMA waits for its own fragment), both.  The lookahead tests of the current Python sources
# on the product build; the B = 1 and batch tests on the combined variant; then same-box A/Bs at B = 8 and B = 1.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5arr
mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T $R/tests/test_gpu_full_api.py $R/tests/test_gpu_ablation.py $R/tests/test_gpu_api.py > $OUT/tests_la.log 2>&1
echo la tests done
PGMI_LIB_PATH=$R/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi/libpgmi_arrpl.so timeout -k 10 600 \
    $T $R/tests/test_gpu_full_batch.py $R/tests/test_gpu_full.py > $OUT/tests_arrpl.log 2>&1
echo variant tests done
timeout -k 10 900 bash $R/tools/ab_variants.sh "arr pl arrpl" 3 b8 $OUT/ab_b8.txt
timeout -k 10 600 bash $R/tools/ab_variants.sh "arr" 3 b1 $OUT/ab_b1.txt
echo done
