#!/bin/bash
# Round 5: does the caller's stream waiting on the side stream slow the side stream's graphed steps
# (tools/probes/stream_probe.py), and the one-wave-per-row split-K residual + norm (pgmi/libpgmi_srnw.so)
# against the default library on the batch-1 bench (prefill ms in the third column).
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5m
mkdir -p $OUT
timeout -k 10 400 python3 -u $R/tools/probes/stream_probe.py > $OUT/stream_probe.txt 2>&1
timeout -k 10 600 bash $R/tools/ab_variants.sh "srnw" 3 b1 $OUT/ab_srnw.txt
echo done
