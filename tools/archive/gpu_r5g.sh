#!/bin/bash
# Round 5: lookahead without the caller-stream hop after hits (tests + drop-in numbers), and the same-box
# B = 8 A/B of the RMSNorm folds against the round-4 library (pgmi/libpgmi_r4.so, built from HEAD).
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5g
mkdir -p $OUT
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T $R/tests/test_gpu_full_api.py $R/tests/test_gpu_full_batch.py > $OUT/tests.log 2>&1
timeout -k 10 600 bash $R/tools/ab_variants.sh "r4" 3 b8 $OUT/ab_b8.txt
for i in 1 2; do
  timeout -k 10 300 python3 -u $R/bench.py --no-448 --no-cpu-baseline --prefill-iters 3 --steps 64 --nokv-tokens 2 \
    > $OUT/bench_$i.json 2> $OUT/bench_$i.err
done
echo done
