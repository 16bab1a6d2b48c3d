#!/bin/bash
# Round 5 closing evidence, second half (tools/archive/gpu_r5final.sh's tests, smoke and bench ran on these sources; its
# MFMA-busy pass crashed in the profiler at start-up, before the program ran): the per-kernel trace and HBM passes
# for this csrc digest (the prefill GEMMs' MFMA-busy record r05_kernel_pmc_mfma.csv predates only decode-GEMV
# changes), then the bench line again with pmc_traffic.json matching the build.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5final3
mkdir -p $OUT
SKIP_MFMA=1 timeout -k 10 900 bash $R/tools/gpu_kernel_pmc.sh r05 > $OUT/kpmc.log 2>&1
echo pmc done
cp $R/gpurun_out/kpmc_r05/pmc_traffic.json $R/profiles/pmc_traffic.json
timeout -k 10 500 python3 -u $R/bench.py > $OUT/bench.json 2> $OUT/bench.err
echo done
