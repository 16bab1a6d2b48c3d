#!/bin/bash
# round 6: B = 1 q|k|v prefetching this layer's cached K / V rows into the Infinity Cache (-DPGMI_KV_PF=1, pgmi/libpgmi.so)
# against the build without it (pgmi/libpgmi_base.so): decode parity tests on the variant, then a same-box A/B
set -o pipefail
mkdir -p gpurun_out/r6kvpf
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_full.py \
  > gpurun_out/r6kvpf/tests.log 2>&1 && echo tests done && \
timeout -k 10 1000 bash tools/ab_bench.sh 4 > gpurun_out/r6kvpf/ab.txt 2>&1 && echo ab done
