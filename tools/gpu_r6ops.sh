#!/bin/bash
# round 6: the op-level GPU tests (the strided GEMM entry among them)
set -o pipefail
mkdir -p gpurun_out/r6ops
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py \
  > gpurun_out/r6ops/tests.log 2>&1 && echo tests done
