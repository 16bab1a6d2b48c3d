#!/bin/bash
# Same-box A/B of two builds of libpgmi (base = pgmi/libpgmi_base.so, new = pgmi/libpgmi.so) on the
# 8-images-per-GPU leg (configs[3]'s per-GPU share: 8-image prefill + B = 8 decode), alternating.
# usage (via gpurun): bash tools/ab_b8.sh [rounds]
set -e
B=$GRAFT_REPO_ROOT/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi/libpgmi_base.so
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/ab
for i in $(seq 1 ${1:-2}); do
  for v in base new; do
    if [ $v = base ]; then export PGMI_LIB_PATH=$B; else unset PGMI_LIB_PATH; fi
    timeout -k 10 300 python $GRAFT_REPO_ROOT/bench.py --steps 32 --warmup 4 --no-448 --no-api --no-cpu-baseline \
      --prefill-iters 5 --nokv-tokens 2 > $GRAFT_REPO_ROOT/gpurun_out/ab/b8.log 2>&1
    echo "$v $(tail -n 1 $GRAFT_REPO_ROOT/gpurun_out/ab/b8.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d["config4_images_per_gpu"]; print(d["prefill_ms"], d["prefill_vision_ms"], c["prefill_ms"], c["ms_per_step"])')"
  done
done
