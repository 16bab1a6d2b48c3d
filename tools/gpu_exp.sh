#!/bin/bash
# Experiment batch on the GPU box: attention parity (ops tests), the prefetch probe, the in-situ
# vision plan sweep.  usage: bash tools/gpu_exp.sh <tag>
set -e
TAG=${1:-exp}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/ops.log 2>&1
echo ops done
timeout -k 10 200 python -u $R/tools/probes/prefetch_probe.py > $OUT/prefetch.log 2>&1
echo prefetch done
timeout -k 10 300 python -u $R/tools/probes/decode_prefetch_sweep.py > $OUT/dpf.log 2>&1
echo decode prefetch done
timeout -k 10 600 python -u $R/tools/probes/vision_plan_sweep.py > $OUT/vsweep.log 2>&1
echo done
