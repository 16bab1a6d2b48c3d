#!/bin/bash
# Round-4: SigLIP LayerNorm2 via out_proj segment statistics (PGMI_VISION_LNFOLD=2, no in-launch hand-off)
# -- its parity test, then the tower time, separate LayerNorm launches (0) vs mode 2.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
PGMI_PARITY_LOG=$O/parity_fold_o.jsonl timeout -k 10 400 python -u -m pytest tests/test_gpu_full.py -x -q \
  -k "lnfold" --timeout 300 --timeout-method thread > $O/t_fold_o.log 2>&1
for i in 1 2; do
  for v in 0 2; do
    PGMI_VISION_LNFOLD=$v timeout -k 10 300 python bench.py --batch 1 --steps 16 --warmup 4 --no-448 --no-extra --no-api \
      --no-cpu-baseline --prefill-iters 30 > $O/vf.log 2>&1
    echo "lnfold=$v $(tail -n 1 $O/vf.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["prefill_vision_ms"], d["prefill_ms"], d["value"])')" >> $O/ab_r4o.txt
  done
done
