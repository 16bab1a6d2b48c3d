#!/bin/bash
# Round-4: non-temporal weight pieces for single-row-tile warp-specialised GEMMs (k_gemm_w, default on;
# PGMI_GEMM_WNT=0 off): the GEMM/model tests touching it, then same-box prefill pairs at 224 px (the
# M = 288 gate|up is the one such GEMM).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model_small.py tests/test_gpu_full.py -x -q \
  --timeout 300 --timeout-method thread -k "gemm or prefill or teacher_forced_64" > $O/t_wnt.log 2>&1
for i in 1 2 3; do
  for v in 0 1; do
    PGMI_GEMM_WNT=$v timeout -k 10 300 python bench.py --steps 16 --warmup 4 --no-448 --no-extra --no-api \
      --no-cpu-baseline --prefill-iters 20 > $O/wnt.log 2>&1
    echo "wnt=$v $(tail -n 1 $O/wnt.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); g=d["prefill_gemm_roofline"]["gate_up_geglu"]; print(d["prefill_ms"], d["prefill_lm_ms"], g["avg_launch_us"], g["isolated"]["avg_launch_us"])')" >> $O/ab_r4l.txt
  done
done
