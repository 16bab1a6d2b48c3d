#!/bin/bash
# PMC passes (tools/gemm_pmc.sh) over several GEMM plans; usage: bash tools/gpu_gemm_pmc.sh <tag> "<shape:cfg:split> ..."
set -e
R=$GRAFT_REPO_ROOT
for spec in $2; do
  IFS=: read -r shape cfg split <<< "$spec"
  bash $R/tools/gemm_pmc.sh ${1}_${shape}_$cfg $shape $cfg $split
  echo "$spec done"
done
