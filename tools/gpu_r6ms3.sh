#!/bin/bash
# round 6: the multi-step decode A/B again on another box (B = 8 and B = 3; tools/probes/multistep_probe.py)
set -o pipefail
mkdir -p gpurun_out/r6ms3
timeout -k 10 300 python -u tools/probes/multistep_probe.py --batch 8 --steps 64 --rounds 4 --ns 8 \
  > gpurun_out/r6ms3/b8.log 2>&1 && \
timeout -k 10 300 python -u tools/probes/multistep_probe.py --batch 3 --steps 64 --rounds 3 --ns 8 \
  > gpurun_out/r6ms3/b3.log 2>&1 && echo probe done
