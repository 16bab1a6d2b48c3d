#!/bin/bash
# Round-4 same-box A/Bs: prefill with the XCD block raster of the GEMMs (PGMI_GEMM_XBLK=1, default)
# vs the run order (=0); B = 8 decode with the attention combine folded (PGMI_FUSED_COMB=1, default)
# vs its own launch (=0); then the HBM probe (FETCH_SIZE / WRITE_SIZE per launch).
# usage (via gpurun): bash tools/archive/gpu_r4c.sh
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
for i in 1 2; do
  for v in 0 1; do
    PGMI_GEMM_XBLK=$v PGMI_FUSED_COMB=$v timeout -k 10 300 python bench.py --steps 64 --warmup 8 --no-api \
      --no-cpu-baseline --prefill-iters 10 --nokv-tokens 2 > $O/ab.log 2>&1
    echo "xblk=comb=$v $(tail -n 1 $O/ab.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d["config4_images_per_gpu"]; print(d["value"], d["prefill_ms"], d["prefill_vision_ms"], d["prefill_448"]["prefill_ms"], d["prefill_448"]["prefill_vision_ms"], c["prefill_ms"], c["ms_per_step"])')" >> $O/ab_r4c.txt
  done
done
[ "$1" = hbm ] && bash tools/gpu_hbm_probe.sh r04 || true
