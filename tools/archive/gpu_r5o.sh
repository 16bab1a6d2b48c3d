#!/bin/bash
# Round 5: the lookahead with the logits copy on the caller's stream after a host wait (no op between two lookaheads) -- drop-in tests,
# the loop's timeline, the bench's drop-in numbers.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5o
mkdir -p $OUT
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T $R/tests/test_gpu_full_api.py $R/tests/test_gpu_ablation.py > $OUT/tests.log 2>&1
timeout -k 10 300 python3 -u $R/tools/probes/lookahead_probe.py > $OUT/lookahead_probe.txt 2>&1
timeout -k 10 300 python3 -u $R/bench.py --no-448 --no-cpu-baseline --prefill-iters 3 --steps 64 --nokv-tokens 2 \
    > $OUT/bench.json 2> $OUT/bench.err
echo done
