#!/bin/bash
# Round 5 closing evidence after the last Python changes (csrc unchanged since tools/archive/gpu_r5final.sh, so its
# per-kernel profile and pmc_traffic.json still match): every -m gpu test with the parity records, smoke(), and
# the default bench line (config4 at 256 steps).  Each step under its own limit.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5final2
mkdir -p $OUT
PGMI_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 \
    --timeout-method thread > $OUT/tests.log 2>&1
echo tests done
timeout -k 10 300 python3 -u -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > $OUT/smoke.log 2>&1
echo smoke done
timeout -k 10 500 python3 -u $R/bench.py > $OUT/bench.json 2> $OUT/bench.err
echo done
