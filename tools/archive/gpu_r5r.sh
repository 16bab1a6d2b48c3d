#!/bin/bash
# Round 5: the gate|up fragment-major image (non-temporal) kept, down row-major -- batched tests (full and small
# models) and the same-box B = 8 A/B against the previous commit's library.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5r
mkdir -p $OUT
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
PGMI_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 400 $T $R/tests/test_gpu_full_batch.py $R/tests/test_gpu_model_small.py > $OUT/tests.log 2>&1
timeout -k 10 600 bash $R/tools/ab_variants.sh "fold" 3 b8 $OUT/ab_b8.txt
echo done
