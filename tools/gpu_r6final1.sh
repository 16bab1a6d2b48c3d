#!/bin/bash
# Round 6 closing evidence, first half (on the final sources): the per-kernel trace of one bench.py run, the
# MFMA-busy pass, the FETCH_SIZE / WRITE_SIZE passes and pmc_traffic.json for this csrc digest
# (tools/gpu_kernel_pmc.sh), each under its own limit.
set -e
R=$GRAFT_REPO_ROOT
timeout -k 10 1100 bash $R/tools/gpu_kernel_pmc.sh r06 > $R/gpurun_out/kpmc_r06.log 2>&1
echo kpmc done
