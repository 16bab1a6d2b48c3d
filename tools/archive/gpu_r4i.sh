#!/bin/bash
# Round-4 probe: the B = 8 lm_head on the streaming v_dot2 GEMV (PGMI_B8_LM_DOT=1) vs the MFMA ring,
# same-box pairs, then the batched parity test with it on.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
for i in 1 2; do
  for v in 0 1; do
    PGMI_B8_LM_DOT=$v timeout -k 10 300 python bench.py --batch 8 --steps 64 --warmup 8 --no-448 --no-extra --no-api \
      --no-cpu-baseline --prefill-iters 3 > $O/b8l.log 2>&1
    echo "lmdot=$v $(tail -n 1 $O/b8l.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab_r4i.txt
  done
done
PGMI_B8_LM_DOT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_full_batch.py -x -q --timeout 300 \
  --timeout-method thread > $O/t_b8lm.log 2>&1
