#!/bin/bash
# round 6: the prefill GEMMs against the operands' row pitch (tools/probes/stride_probe.py)
set -o pipefail
mkdir -p gpurun_out/r6st
timeout -k 10 600 python -u tools/probes/stride_probe.py --rounds 3 > gpurun_out/r6st/stride.log 2>&1 && echo stride done
