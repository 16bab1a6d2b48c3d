#!/bin/bash
# Round-4 same-box A/Bs of the B = 1 decode step: the small projections' weights read with the
# temporal load (libpgmi.so, PGMI_SMALL_NT=1) vs the streaming load (libpgmi_smallt.so), and the
# o_proj workgroup cap (PGMI_ORES_CAP 256 default vs 128 / 64); then the default prefill/batched line
# with the XCD block raster limited to >= 2048-row GEMMs and the combine launch unfolded.
# usage (via gpurun): bash tools/archive/gpu_r4d.sh
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
bash tools/ab_variants.sh "smallt" 2 b1 $O/ab_r4d.txt
for i in 1 2; do
  for c in 256 128 64; do
    PGMI_ORES_CAP=$c timeout -k 10 300 python bench.py --steps 256 --warmup 16 --no-448 --no-extra --no-api \
      --no-cpu-baseline --prefill-iters 3 > $O/abc.log 2>&1
    echo "cap=$c $(tail -n 1 $O/abc.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab_r4d.txt
  done
done
for v in 0 1; do
  PGMI_GEMM_XBLK=$v timeout -k 10 300 python bench.py --steps 64 --warmup 8 --no-api \
    --no-cpu-baseline --prefill-iters 10 --nokv-tokens 2 > $O/ab.log 2>&1
  echo "xblk=$v $(tail -n 1 $O/ab.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d["config4_images_per_gpu"]; print(d["value"], d["prefill_ms"], d["prefill_vision_ms"], d["prefill_448"]["prefill_ms"], d["prefill_448"]["prefill_vision_ms"], c["prefill_ms"], c["ms_per_step"])')" >> $O/ab_r4d.txt
done
