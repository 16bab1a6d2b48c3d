#!/bin/bash
# Kernel trace + SQ PMC passes over the prefill-attention probe (tools/probes/attn_bench.py <variants>):
# pass 1 issue/wait mix, pass 2 LDS traffic and MFMA busy.
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
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/pmc2 -o run -- python3 -u $R/tools/probes/attn_bench.py $2 > $OUT/pmc2.log 2>&1
echo pmc2 done
