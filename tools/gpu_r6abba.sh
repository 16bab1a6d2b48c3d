#!/bin/bash
# round 6: A/A (two copies of the HEAD build: the A/B method's own spread and order effects), then HEAD against the
# lm_head fold with its partials loaded up front, both in balanced order (tools/ab_abba.sh)
set -o pipefail
P=$GRAFT_REPO_ROOT/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi
mkdir -p gpurun_out/r6abba
bash tools/ab_abba.sh $P/libpgmi.so $P/libpgmi_aa.so 2 > gpurun_out/r6abba/aa.txt 2>&1 && echo aa done && \
bash tools/ab_abba.sh $P/libpgmi.so $P/libpgmi_fold.so 3 > gpurun_out/r6abba/fold.txt 2>&1 && echo fold done
