#!/bin/bash
# Round 5: the batched decode's RMSNorm folds (o_proj / down epilogues write partial sums of squares, gate|up and
# q|k|v normalise on load; the down projection's combine in-launch) and the drop-in lookahead: their GPU tests
# first, then the rest of the suite with parity records (PGMI_PARITY_LOG), then the bench line.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5f
mkdir -p $OUT
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
PGMI_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 400 $T $R/tests/test_gpu_full_batch.py $R/tests/test_gpu_full_api.py > $OUT/first.log 2>&1
PGMI_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 900 $T -m gpu $R/tests --ignore=$R/tests/test_gpu_full_batch.py --ignore=$R/tests/test_gpu_full_api.py > $OUT/tests.log 2>&1
timeout -k 10 500 python3 -u $R/bench.py > $OUT/bench.json 2> $OUT/bench.err
echo done
