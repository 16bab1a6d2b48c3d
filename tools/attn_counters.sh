#!/bin/bash
# Counter passes over the prefill attention kernels in isolation (tools/probes/attn_bench.py on one
# shape), each rocprofv3 --pmc pass under its own limit.  usage (via gpurun): bash tools/attn_counters.sh <tag> <shape> <variants...>
set -e
TAG=${1:-ac}; SH=$2; shift 2
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export ATTN_SHAPES=$SH
P="python3 $R/tools/probes/attn_bench.py $@"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $P > $OUT/trace.log 2>&1
echo trace done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/sq -o run -- $P > $OUT/sq.log 2>&1
echo sq done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH \
    --output-format csv -d $OUT/sq2 -o run -- $P > $OUT/sq2.log 2>&1
echo sq2 done
