#!/bin/bash
# Round 5: what slows the graphed step on a non-blocking side stream (tools/probes/stream_probe.py, same-process
# baselines), then the one-wave-per-row split-K residual + norm (pgmi/libpgmi_srnw.so) against the default
# library on the batch-1 bench (prefill ms in the third column).
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5l
mkdir -p $OUT
timeout -k 10 400 python3 -u $R/tools/probes/stream_probe.py > $OUT/stream_probe.txt 2>&1
if [ -f $R/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi/libpgmi_srnw.so ]; then
  timeout -k 10 600 bash $R/tools/ab_variants.sh "srnw" 3 b1 $OUT/ab_srnw.txt
fi
echo done
