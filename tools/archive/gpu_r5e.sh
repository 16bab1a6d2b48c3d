#!/bin/bash
# Round 5: the drop-in lookahead on a side stream -- its GPU tests, then the bench line (dropin_api with and
# without it), parity records of every model-level test (PGMI_PARITY_LOG) for DESIGN sec.5's table.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5e
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_full_api.py -x -v --timeout 300 --timeout-method thread > $OUT/api.log 2>&1
PGMI_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
timeout -k 10 500 python3 -u $R/bench.py > $OUT/bench.json 2> $OUT/bench.err
echo done
