#!/bin/bash
# Round-4: B = 1 down projection, bytes in flight per CU: workgroup cap x rows in flight per wave
# (PGMI_DOWN_CAP / PGMI_DOWN_DEPTH: probe knobs of that build, removed after this A/B kept the default
# 512 x 1), same box, two alternating rounds; record profiles/r04_down_inflight_ab.txt.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
for i in 1 2; do
  for v in "512 1" "1024 1" "512 2" "256 2"; do
    set -- $v
    PGMI_DOWN_CAP=$1 PGMI_DOWN_DEPTH=$2 timeout -k 10 300 python bench.py --batch 1 --steps 256 --warmup 16 --no-448 \
      --no-extra --no-api --no-cpu-baseline --prefill-iters 3 > $O/dn.log 2>&1
    echo "cap=$1 depth=$2 $(tail -n 1 $O/dn.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab_r4p.txt
  done
done
