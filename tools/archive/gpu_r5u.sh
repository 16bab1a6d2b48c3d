#!/bin/bash
# Round 5: (1) the down projection from a fragment-major image with one-deep streams (probe build libpgmi_dn1.so)
# against the default, B = 8; (2) HIP runtime settings for kernel arguments / graph packets, B = 1 and B = 8.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5u
mkdir -p $OUT
timeout -k 10 600 bash $R/tools/ab_variants.sh "dn1" 3 b8 $OUT/ab_b8.txt
timeout -k 10 900 bash $R/tools/b8_env.sh 2 "HIP_FORCE_DEV_KERNARG=1" "DEBUG_HIP_GRAPH_PACKET_CAPTURE=1" \
    "DEBUG_HIP_GRAPH_PACKET_CAPTURE=0" > $OUT/env.txt 2>&1
echo done
