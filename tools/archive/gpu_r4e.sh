#!/bin/bash
# Round-4 probe: B = 1 decode with part of each layer's gate|up weights read into the Infinity Cache
# ahead of the GEGLU GEMV (PGMI_PF, engine.hip pf_cfg): serial (1) and on a forked side stream (2)
# at several fractions / grid sizes, then kernel traces of PF=1 and PF=2 (timestamps show overlap).
# usage (via gpurun): bash tools/archive/gpu_r4e.sh
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
run() {  # label, env...
  local l=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 256 --warmup 16 --no-448 --no-extra --no-api \
    --no-cpu-baseline --prefill-iters 3 > $O/pf.log 2>&1
  echo "$l $(tail -n 1 $O/pf.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab_r4e.txt
}
for i in 1 2; do
  run base PGMI_PF=0
  run serial8 PGMI_PF=1 PGMI_PF_Q=8
  run br4w256 PGMI_PF=2 PGMI_PF_Q=4 PGMI_PF_WG=256
  run br8w256 PGMI_PF=2 PGMI_PF_Q=8 PGMI_PF_WG=256
  run br4w64 PGMI_PF=2 PGMI_PF_Q=4 PGMI_PF_WG=64
  run br6w128 PGMI_PF=2 PGMI_PF_Q=6 PGMI_PF_WG=128
  run br2w128 PGMI_PF=2 PGMI_PF_Q=2 PGMI_PF_WG=128
done
export TMPDIR=/tmp
for m in 1 2; do
  PGMI_PF=$m PGMI_PF_Q=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pf$m -o pf -- python3 bench.py \
    --steps 32 --warmup 4 --no-448 --no-extra --no-api --no-cpu-baseline --prefill-iters 1 > $O/pfprof$m.log 2>&1
done
