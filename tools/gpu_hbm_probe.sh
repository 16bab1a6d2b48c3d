#!/bin/bash
# HBM bytes per launch of every kernel of the short PMC probe (one 224 px prefill + eager decode at
# B = 1, then the 8-image batch prefill + decode at B = 8): kernel trace, FETCH_SIZE and WRITE_SIZE
# in separate passes, summary by tools/kernel_pmc.py (FETCH_SIZE doubled: MI355X_MICROARCH.md HBM).
# The tail of tools/gpu_kernel_pmc.sh without its whole-bench trace and MFMA pass.
# usage (from the repo root, via gpurun): bash tools/gpu_hbm_probe.sh <tag>
set -e
TAG=${1:-probe}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/hbm_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P="python3 $R/tools/probes/pmc_probe.py 3"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/ptrace -o run -- $P > $OUT/ptrace.log 2>&1
echo probe trace done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $P > $OUT/fetch.log 2>&1
echo fetch done
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $P > $OUT/write.log 2>&1
echo write done
python3 $R/tools/kernel_pmc.py $OUT/ptrace/run_kernel_trace.csv - \
    $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv $OUT/kernel_hbm_probe.csv > $OUT/summary.txt
echo done
