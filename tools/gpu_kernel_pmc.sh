#!/bin/bash
# Per-kernel evidence of one bench.py run (every config leg: 224/448 prefill, B = 1 and B = 8 decode):
# kernel-trace stats, then MFMA-busy (SQ + GRBM), FETCH_SIZE and WRITE_SIZE in separate --pmc passes,
# each step under its own limit; summary by tools/kernel_pmc.py.
# usage (from the repo root, via gpurun): bash tools/gpu_kernel_pmc.sh <tag>
set -e
TAG=${1:-r02}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/kpmc_$TAG
mkdir -p $OUT
# heartbeat: a pass can run past gpurun's 180 s silence limit without printing
( while true; do date +%s >> $OUT/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 16 --warmup 4 --no-cpu-baseline --no-api --prefill-iters 3 --kernel-iters 18 --nokv-tokens 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py $ARGS > $OUT/trace.log 2>&1
echo trace done
# FETCH_SIZE / WRITE_SIZE and the MFMA-busy pass over the short probe (prefill + eager decode, B = 1 and 8, and
# the 448 px prefill): a TCC pass over bench.py's every-leg run does not finish, and (round 6) the SQ pass over
# bench.py's graphed decode steps crashed the profiled process in hipGraph capture (host SIGSEGV in decode_step)
P="python3 $R/tools/probes/pmc_probe.py 3 448"
# SKIP_MFMA=1: keep the trace + HBM passes only
if [ "${SKIP_MFMA:-0}" != 1 ]; then
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/mfma -o run -- $P > $OUT/mfma.log 2>&1
echo mfma done
fi
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/ptrace -o run -- $P > $OUT/ptrace.log 2>&1
echo probe trace done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $P > $OUT/fetch.log 2>&1
echo fetch done
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $P > $OUT/write.log 2>&1
echo write done
M=-
[ "${SKIP_MFMA:-0}" != 1 ] && M=$OUT/mfma/run_counter_collection.csv
python3 $R/tools/kernel_pmc.py $OUT/ptrace/run_kernel_trace.csv $M \
    $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv $OUT/kernel_hbm_probe.csv > $OUT/summary.txt
echo done
PGMI_ROUND=$TAG python3 $R/tools/pmc_traffic.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv \
    "k_gemv<1, 4, 1, 2, 1, true, 1, false>" gateup $OUT/pmc_traffic.json >> $OUT/summary.txt
echo traffic done
python3 $R/tools/prefill_gemm_shapes.py $OUT/trace/run_kernel_trace.csv $OUT/prefill_gemm_shapes.csv >> $OUT/summary.txt
echo shapes done
