#!/bin/bash
# Round profile on the GPU box: kernel-trace stats of bench.py, then FETCH_SIZE and WRITE_SIZE
# in separate --pmc passes (MI355X_MICROARCH.md: TCC slots), each step under its own limit.
# usage (from the repo root, via gpurun): bash tools/gpu_profile.sh <round-tag>
set -e
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 64 --warmup 8 --no-cpu-baseline --prefill-iters 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py $ARGS > $OUT/bench_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
    python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline --prefill-iters 1 --kernel-iters 18 > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
    python3 $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline --prefill-iters 1 --kernel-iters 18 > $OUT/write.log 2>&1
echo done
