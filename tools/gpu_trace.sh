#!/bin/bash
# Kernel-trace stats of a short bench.py run (224 px prefill + B=1 decode only) on the GPU box.
# usage (from the repo root, via gpurun): bash tools/gpu_trace.sh <tag> [extra bench args]
set -e
TAG=${1:-trace}
shift || true
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py --steps 64 --warmup 8 --no-cpu-baseline --prefill-iters 5 --no-448 --no-extra --no-api "$@" \
    > $OUT/bench_trace.log 2>&1
echo done
