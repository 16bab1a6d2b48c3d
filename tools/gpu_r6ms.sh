#!/bin/bash
# round 6: one-launch-per-step decode against n steps per hipGraph launch (pgmi_decode_steps), B = 1 and 8
set -o pipefail
mkdir -p gpurun_out/r6ms
timeout -k 10 300 python -u tools/probes/multistep_probe.py --batch 1 --steps 64 --rounds 4 --ns 4,8,16 \
  > gpurun_out/r6ms/b1.log 2>&1 && \
timeout -k 10 300 python -u tools/probes/multistep_probe.py --batch 8 --steps 64 --rounds 3 --ns 4,8,16 \
  > gpurun_out/r6ms/b8.log 2>&1 && echo probe done
