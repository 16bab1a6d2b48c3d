#!/bin/bash
# Counter study of the M = 288 text GEMMs (gate|up + GeGLU, down split 8) in isolation: separate
# rocprofv3 --pmc passes (SQ + GRBM; TA/TCP/TCC) over tools/gemm_sweep.py's cold calls, each pass
# under its own limit.  usage (via gpurun): bash tools/gemm_counters.sh <tag>
set -e
TAG=${1:-gc}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P="python3 $R/tools/gemm_sweep.py t_gateup t_down --cold --cfgs 31 --splits 8 --iters 20"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- $P > $OUT/trace.log 2>&1
echo trace done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/sq -o run -- $P > $OUT/sq.log 2>&1
echo sq done
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum \
    --output-format csv -d $OUT/mem -o run -- $P > $OUT/mem.log 2>&1
echo mem done
