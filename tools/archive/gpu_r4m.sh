#!/bin/bash
# Round-4: B = 8 decode, staged (default) vs unstaged MFMA projections after the cache-policy change.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
for i in 1 2; do
  for v in 1 0; do
    PGMI_MF_STAGED=$v timeout -k 10 300 python bench.py --batch 8 --steps 64 --warmup 8 --no-448 --no-extra --no-api \
      --no-cpu-baseline --prefill-iters 3 > $O/st.log 2>&1
    echo "staged=$v $(tail -n 1 $O/st.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab_r4m.txt
  done
done
