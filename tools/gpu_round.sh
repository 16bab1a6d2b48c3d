#!/bin/bash
# Round-end evidence on the GPU box: GPU parity tests, the default bench line (cpu_baseline
# included), and a rocprofv3 kernel-trace summary of a shorter bench run; each step bounded.
# usage (from the repo root, via gpurun): bash tools/gpu_round.sh <tag>
set -e
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/round_$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
timeout -k 10 400 python3 -u $R/bench.py > $OUT/bench.json 2> $OUT/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py --steps 64 --warmup 8 --no-cpu-baseline --prefill-iters 5 > $OUT/bench_trace.log 2>&1
echo done
