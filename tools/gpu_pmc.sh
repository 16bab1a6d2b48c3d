#!/bin/bash
# HBM traffic passes (FETCH_SIZE, WRITE_SIZE: separate --pmc runs, MI355X_MICROARCH.md HBM section)
# over a short decode-only bench run, each under its own limit.
# usage (from the repo root, via gpurun): bash tools/gpu_pmc.sh <tag>
set -e
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 8 --warmup 2 --no-cpu-baseline --no-448 --no-extra --prefill-iters 1 --kernel-iters 18"
timeout -k 10 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py $ARGS > $OUT/fetch.log 2>&1
echo fetch done
timeout -k 10 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $R/bench.py $ARGS > $OUT/write.log 2>&1
echo write done
