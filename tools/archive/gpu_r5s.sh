#!/bin/bash
# Round 5: the batched lm_head on MFMA over E's fragment-major image (1,024 / 512 / 2,048 workgroups) against the
# previous commit's LDS-DMA ring (libpgmi_img.so), same box, B = 8; batch tests of the default build first.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5s
mkdir -p $OUT
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
PGMI_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 400 $T $R/tests/test_gpu_full_batch.py $R/tests/test_gpu_model_small.py > $OUT/tests.log 2>&1
timeout -k 10 900 bash $R/tools/ab_variants.sh "img lm512 lm2048" 3 b8 $OUT/ab_b8.txt
echo done
