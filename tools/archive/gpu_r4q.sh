#!/bin/bash
# Round-4: B = 8 gate|up workgroups for the (now default) unstaged form with the default cache policy
# (PGMI_MF_GU_BLOCKS), same box, two alternating rounds.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
for i in 1 2; do
  for v in 512 1024 768 384; do
    PGMI_MF_GU_BLOCKS=$v timeout -k 10 300 python bench.py --batch 8 --steps 64 --warmup 8 --no-448 --no-extra --no-api \
      --no-cpu-baseline --prefill-iters 3 > $O/gu.log 2>&1
    echo "gu_blocks=$v $(tail -n 1 $O/gu.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab_r4q.txt
  done
done
