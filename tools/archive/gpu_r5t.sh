#!/bin/bash
# Round 5: fragment-major images for the batched q|k|v (in its row order) and o_proj GEMVs too -- batched tests, the
# same-box B = 8 A/B against the previous commit (gate|up image only, libpgmi_img.so), kernel stats.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5t
mkdir -p $OUT
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
PGMI_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 400 $T $R/tests/test_gpu_full_batch.py $R/tests/test_gpu_model_small.py > $OUT/tests.log 2>&1
timeout -k 10 600 bash $R/tools/ab_variants.sh "img" 3 b8 $OUT/ab_b8.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 $R/bench.py --batch 8 --steps 64 --warmup 8 --no-448 --no-extra --no-api --no-cpu-baseline --prefill-iters 3 \
    > $OUT/prof.log 2>&1
echo done
