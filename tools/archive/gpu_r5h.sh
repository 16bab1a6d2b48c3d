#!/bin/bash
# Round 5: why the batched RMSNorm folds and the side-stream lookahead did not pay: kernel-trace stats of the
# B = 8 step for this build and the round-4 library (pgmi/libpgmi_r4.so), and the drop-in loop's timeline
# (tools/probes/lookahead_probe.py).
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5h
mkdir -p $OUT
timeout -k 10 300 python3 -u $R/tools/probes/lookahead_probe.py > $OUT/lookahead_probe.txt 2>&1
cd /tmp && export TMPDIR=/tmp
ARGS="--batch 8 --steps 64 --warmup 8 --no-448 --no-extra --no-api --no-cpu-baseline --prefill-iters 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/new -o run -- \
    python3 $R/bench.py $ARGS > $OUT/new.log 2>&1
export PGMI_LIB_PATH=$R/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi/libpgmi_r4.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r4 -o run -- \
    python3 $R/bench.py $ARGS > $OUT/r4.log 2>&1
echo done
