#!/bin/bash
# Round-4: 448 px decode parity (new fixture), then B = 8 decode on v_dot2 GEMVs over RMSNorm'd rows
# (PGMI_B8_DOT=1, PGMI_MF_STAGED=0) vs the MFMA kernels: same-box bench pairs and the batched parity test.
# usage (via gpurun): bash tools/archive/gpu_r4h.sh
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
PGMI_PARITY_LOG=$O/parity_448.jsonl timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py -k "448" -x -v \
  --timeout 300 --timeout-method thread > $O/t448.log 2>&1
for i in 1 2; do
  for v in 0 1; do
    PGMI_MF_STAGED=$v PGMI_B8_DOT=$((1 - v)) timeout -k 10 300 python bench.py --batch 8 --steps 64 --warmup 8 \
      --no-448 --no-extra --no-api --no-cpu-baseline --prefill-iters 3 > $O/b8d.log 2>&1
    echo "staged=$v dot=$((1 - v)) $(tail -n 1 $O/b8d.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab_r4h.txt
  done
done
PGMI_MF_STAGED=0 PGMI_B8_DOT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_full_batch.py -x -q \
  --timeout 300 --timeout-method thread > $O/t_b8dot.log 2>&1
