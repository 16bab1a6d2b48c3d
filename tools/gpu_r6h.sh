#!/bin/bash
# Round 6: every -m gpu test (the regenerated 1,024-sample batch fixtures, the drop-in loop's per-step parity,
# the M = 288 down projection on W288n split 8) with parity records, smoke, the bench line
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6h
mkdir -p $OUT
PGMI_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 \
    --timeout-method thread > $OUT/tests.log 2>&1
echo tests done
timeout -k 10 300 python3 -u -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > $OUT/smoke.log 2>&1
echo smoke done
timeout -k 10 500 python3 -u $R/bench.py --steps 20 > $OUT/bench.json 2> $OUT/bench.err
echo bench done
