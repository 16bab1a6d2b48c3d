#!/bin/bash
# Round 6 closing evidence, second half: every -m gpu test with the parity records, smoke(), then the bench line
# with profiles/pmc_traffic.json (from tools/gpu_r6final1.sh, same csrc digest) in place.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6final
mkdir -p $OUT
PGMI_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 \
    --timeout-method thread > $OUT/tests.log 2>&1
echo tests done
timeout -k 10 300 python3 -u -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > $OUT/smoke.log 2>&1
echo smoke done
timeout -k 10 500 python3 -u $R/bench.py --steps 20 > $OUT/bench.json 2> $OUT/bench.err
echo bench done
