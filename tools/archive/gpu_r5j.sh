#!/bin/bash
# Round 5: the graphed decode step on streams other than the caller's default one (tools/probes/stream_probe.py),
# and a kernel trace of the batch-1 bench (vision tower / prefill launches) for the round's profile.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5j
mkdir -p $OUT
timeout -k 10 400 python3 -u $R/tools/probes/stream_probe.py > $OUT/stream_probe.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/b1 -o run -- \
    python3 $R/bench.py --steps 64 --warmup 8 --no-448 --no-extra --no-api --no-cpu-baseline --prefill-iters 5 > $OUT/b1.log 2>&1
echo done
