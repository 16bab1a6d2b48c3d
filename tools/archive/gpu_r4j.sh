#!/bin/bash
# Round-4: stream-K tail split of the 8-phase GEMM (PGMI_GEMM_SK, default on): GEMM op tests and the 448 px
# / batched parity tests, then same-box prefill pairs (448 px, 8 images) with it off / on.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_full.py tests/test_gpu_full_batch.py -x -q \
  --timeout 300 --timeout-method thread -k "gemm or 448 or batch" > $O/t_sk.log 2>&1
for i in 1 2; do
  for v in 0 1; do
    PGMI_GEMM_SK=$v timeout -k 10 300 python bench.py --steps 16 --warmup 4 --no-api --no-cpu-baseline \
      --prefill-iters 10 --nokv-tokens 2 > $O/sk.log 2>&1
    echo "sk=$v $(tail -n 1 $O/sk.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d["config4_images_per_gpu"]; g=d["prefill_448"]["gemm_roofline"]["gate_up_geglu"]; print(d["prefill_ms"], d["prefill_448"]["prefill_ms"], c["prefill_ms"], g["avg_launch_us"], g["isolated"]["avg_launch_us"])')" >> $O/ab_r4j.txt
  done
done
