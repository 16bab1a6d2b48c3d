#!/bin/bash
# Kernel trace + SQ PMC pass over the prefill-attention probe (tools/probes/attn_bench.py <variants>).
# usage: bash tools/gpu_attn_prof.sh <tag> "<variants>"
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 -u $R/tools/probes/attn_bench.py $2 > $OUT/trace.log 2>&1
echo trace done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/pmc -o run -- python3 -u $R/tools/probes/attn_bench.py $2 > $OUT/pmc.log 2>&1
echo pmc done
