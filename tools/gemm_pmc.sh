#!/bin/bash
# PMC passes over one GEMM plan (tools/gemm_pmc.py); usage: bash tools/gemm_pmc.sh <tag> <shape> <cfg> <split>
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM_RD --output-format csv -d $OUT/p1 -o run -- python3 $R/tools/gemm_pmc.py $2 $3 $4 > $OUT/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES --output-format csv -d $OUT/p2 -o run -- python3 $R/tools/gemm_pmc.py $2 $3 $4 > $OUT/p2.log 2>&1
echo ok
