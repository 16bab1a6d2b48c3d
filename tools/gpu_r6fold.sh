#!/bin/bash
# round 6: the lm_head's folded argmax with every partial loaded before the compares -- B <= 2 parity tests on
# the new build, then a same-box A/B of decode against the previous build (pgmi/libpgmi_base.so)
set -o pipefail
mkdir -p gpurun_out/r6fold
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_model_small.py tests/test_gpu_full.py tests/test_gpu_api.py > gpurun_out/r6fold/tests.log 2>&1 && \
echo tests done && timeout -k 10 900 bash tools/ab_bench.sh 3 > gpurun_out/r6fold/ab.txt 2>&1 && echo ab done
