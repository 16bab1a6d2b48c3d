#!/bin/bash
# round 6: pgmi_decode_steps tests (small model: eager / graph, B = 1 / 3) and the batched generate goldens
set -o pipefail
mkdir -p gpurun_out/r6ms2
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_model_small.py tests/test_gpu_full_batch.py tests/test_gpu_full.py \
  > gpurun_out/r6ms2/tests.log 2>&1 && echo tests done && \
timeout -k 10 600 python -u bench.py --steps 20 --warmup 16 --no-cpu-baseline --no-api --no-448 \
  > gpurun_out/r6ms2/bench.log 2>&1 && echo bench done
