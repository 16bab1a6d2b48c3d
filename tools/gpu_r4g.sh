#!/bin/bash
# Round-4: the one-launch MLP half (PGMI_PERSIST=1, kernels_persist.hip) at B = 1 -- numerics against
# the launch path (tools/probes/persist_check.py), then same-box bench pairs.  Each GPU step is
# bounded; the persistent kernel's own waits give up after 20 ms.
# usage (via gpurun): bash tools/gpu_r4g.sh [bench]
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
PGMI_PERSIST=0 timeout -k 10 240 python -u tools/probes/persist_check.py $O/pc0.npz > $O/pc0.log 2>&1
PGMI_PERSIST=1 PGMI_PERSIST_DBG=1 timeout -k 10 240 python -u tools/probes/persist_check.py $O/pc1.npz > $O/pc1.log 2>&1
python tools/probes/persist_check.py --compare $O/pc1.npz $O/pc0.npz > $O/pc_cmp.log 2>&1 || true
cat $O/pc1.log $O/pc_cmp.log
if [ "$1" = bench ]; then
  for i in 1 2 3; do
    for v in 0 1; do
      PGMI_PERSIST=$v timeout -k 10 300 python bench.py --steps 256 --warmup 16 --no-448 --no-extra --no-api \
        --no-cpu-baseline --prefill-iters 3 > $O/pb.log 2>&1
      echo "persist=$v $(tail -n 1 $O/pb.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab_r4g.txt
    done
  done
  export TMPDIR=/tmp
  PGMI_PERSIST=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pp -o pp -- python3 bench.py \
    --steps 32 --warmup 4 --no-448 --no-extra --no-api --no-cpu-baseline --prefill-iters 1 > $O/ppprof.log 2>&1
fi
