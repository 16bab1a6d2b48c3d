#!/bin/bash
# GEMM plan sweep on the GPU box (tools/gemm_sweep.py), output streamed to gpurun_out/<tag>/sweep.txt.
# usage: bash tools/gpu_sweep.sh <tag> "<shapes>" <cfgs> <splits> [--cold ...]
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
timeout -k 10 500 python3 -u $R/tools/gemm_sweep.py $2 --cfgs $3 --splits $4 ${@:5} > $OUT/sweep.txt 2>&1
echo done
