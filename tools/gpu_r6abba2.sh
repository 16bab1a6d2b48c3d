#!/bin/bash
# round 6: HEAD against the lm_head fold with its partials loaded up front, in both balanced orders
# (A B B A and B A A B, three rounds each: tools/ab_abba.sh), so a position effect cancels
set -o pipefail
P=$GRAFT_REPO_ROOT/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi
mkdir -p gpurun_out/r6abba2
bash tools/ab_abba.sh $P/libpgmi.so $P/libpgmi_fold.so 3 > gpurun_out/r6abba2/abba.txt 2>&1 && echo abba done && \
bash tools/ab_abba.sh $P/libpgmi_fold.so $P/libpgmi.so 3 > gpurun_out/r6abba2/baab.txt 2>&1 && echo baab done
