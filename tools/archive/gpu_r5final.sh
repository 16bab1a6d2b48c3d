#!/bin/bash
# Round 5 closing evidence (run on the final sources): every -m gpu test with the parity records, smoke(), the
# default bench line, then the per-kernel profile (tools/gpu_kernel_pmc.sh: kernel trace, MFMA-busy, FETCH_SIZE and
# WRITE_SIZE passes, pmc_traffic.json for this csrc digest).  Each step under its own limit.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5final
mkdir -p $OUT
PGMI_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 \
    --timeout-method thread > $OUT/tests.log 2>&1
echo tests done
timeout -k 10 300 python3 -u -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > $OUT/smoke.log 2>&1
echo smoke done
timeout -k 10 500 python3 -u $R/bench.py > $OUT/bench.json 2> $OUT/bench.err
echo bench done
SKIP_MFMA=${SKIP_MFMA:-0} timeout -k 10 1000 bash $R/tools/gpu_kernel_pmc.sh r05 > $OUT/kpmc.log 2>&1
echo done
