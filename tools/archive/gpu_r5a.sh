#!/bin/bash
# Round 5: GPU parity tests after the cleanup (LayerNorm-fold / fused-combine paths removed, env knobs gone,
# GemmaForCausalLM mask contract, configs[2] / ablation per-step rule), then the default bench line.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5a
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/tests.log 2>&1
timeout -k 10 400 python3 -u $R/bench.py > $OUT/bench.json 2> $OUT/bench.err
echo done
