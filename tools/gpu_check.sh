#!/bin/bash
# Iteration loop on the GPU box: GPU parity tests, then a short kernel-trace profile of bench.py.
# usage (from the repo root, via gpurun): bash tools/gpu_check.sh <tag> [pytest -k expr]
set -e
TAG=${1:-iter}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$2" ]; then K="-k $2"; else K=""; fi
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread $K > $OUT/tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py --steps 64 --warmup 8 --no-cpu-baseline --prefill-iters 5 > $OUT/bench.log 2>&1
timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline > $OUT/bench_plain.log 2>&1
echo done
