#!/bin/bash
# Experiment batch on the GPU box: ops parity tests, then the in-situ plan sweep of the Gemma
# prefill GEMMs.  usage: bash tools/gpu_exp.sh <tag> [plan_sweep args]
set -e
TAG=${1:-exp}
shift || true
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/ops.log 2>&1
echo ops done
timeout -k 10 900 python -u $R/tools/probes/plan_sweep.py "$@" > $OUT/sweep.log 2>&1
echo done
