#!/bin/bash
# The every-leg MFMA-busy PMC pass of tools/gpu_kernel_pmc.sh on its own, with a longer limit (it can
# outlast 240 s on a slow box), against a kernel trace of the same command; summary by tools/kernel_pmc.py.
# usage (from the repo root, via gpurun): bash tools/gpu_mfma_pass.sh <tag>
set -e
TAG=${1:-r04}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/kmfma_$TAG
mkdir -p $OUT
( while true; do date +%s >> $OUT/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 16 --warmup 4 --no-cpu-baseline --no-api --prefill-iters 3 --kernel-iters 18 --nokv-tokens 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py $ARGS > $OUT/trace.log 2>&1
echo trace done
timeout -s KILL 540 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/mfma -o run -- python3 $R/bench.py $ARGS > $OUT/mfma.log 2>&1
echo mfma done
python3 $R/tools/kernel_pmc.py $OUT/trace/run_kernel_trace.csv $OUT/mfma/run_counter_collection.csv \
    - - $OUT/kernel_pmc_bench.csv > $OUT/summary.txt
echo done
