#!/bin/bash
# Round 5: fragment-major images with non-temporal loads -- both GEMVs (base) / gate|up only (libpgmi_gu.so) against
# the previous commit's library (libpgmi_fold.so), same box, B = 8; batch tests of the base build first.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5q
mkdir -p $OUT
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T $R/tests/test_gpu_full_batch.py > $OUT/tests.log 2>&1
timeout -k 10 900 bash $R/tools/ab_variants.sh "fold gu" 3 b8 $OUT/ab_b8.txt
echo done
