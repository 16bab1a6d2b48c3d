#!/bin/bash
# Round 5: the gate|up RMSNorm fold alone (o_proj's epilogue writes the partial sums of squares, k_rows_norm
# gone) -- batch tests and the same-box B = 8 A/B against the round-4 library; the decode step's speed on a
# side stream and with the lookahead's rotating buffers (tools/probes/stream_probe.py).
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5i
mkdir -p $OUT
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
PGMI_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 300 $T $R/tests/test_gpu_full_batch.py > $OUT/tests.log 2>&1
timeout -k 10 300 python3 -u $R/tools/probes/stream_probe.py > $OUT/stream_probe.txt 2>&1
timeout -k 10 600 bash $R/tools/ab_variants.sh "r4" 3 b8 $OUT/ab_b8.txt
echo done
