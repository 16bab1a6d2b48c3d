#!/bin/bash
# round 6: the drop-in loop and the ablation harness timed alone, three rounds (tools/probes/api_probe.py)
set -o pipefail
mkdir -p gpurun_out/r6api
timeout -k 10 600 python -u tools/probes/api_probe.py --rounds 3 > gpurun_out/r6api/api.log 2>&1 && echo api done
