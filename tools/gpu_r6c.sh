#!/bin/bash
# Round 6: the default bench line (with the 256-token configs[1] leg)
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6c
mkdir -p $OUT
timeout -k 10 500 python3 -u $R/bench.py --steps 20 > $OUT/bench.json 2> $OUT/bench.err
echo bench done
