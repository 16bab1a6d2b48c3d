#!/bin/bash
# Round-4 same-box sweep of the B = 1 streaming GEMVs: grid caps and two weight groups in flight
# (PGMI_B1_<GU|DN|LM>_<CAP|D2>, kernels_gemv.hip), then the full-size teacher-forced parity test
# with every two-deep form on.
# usage (via gpurun): bash tools/archive/gpu_r4f.sh
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
run() {  # label, env...
  local l=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 256 --warmup 16 --no-448 --no-extra --no-api \
    --no-cpu-baseline --prefill-iters 3 > $O/sw.log 2>&1
  echo "$l $(tail -n 1 $O/sw.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab_r4f.txt
}
for i in 1 2; do
  run base X=0
  run gu_d2 PGMI_B1_GU_D2=1
  run gu_cap2048 PGMI_B1_GU_CAP=2048
  run gu_cap512 PGMI_B1_GU_CAP=512
  run dn_d2 PGMI_B1_DN_D2=1
  run dn_cap1024 PGMI_B1_DN_CAP=1024
  run dn_cap256 PGMI_B1_DN_CAP=256
  run lm_d2 PGMI_B1_LM_D2=1
  run lm_cap1024 PGMI_B1_LM_CAP=1024
  run lm_cap1536 PGMI_B1_LM_CAP=1536
done
PGMI_B1_GU_D2=1 PGMI_B1_DN_D2=1 PGMI_B1_LM_D2=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py \
  -k teacher_forced_64 -x -q --timeout 300 --timeout-method thread > $O/sw_test.log 2>&1
# speculative K/V issue in the decode attention (default) vs the step-state-first order
bash tools/ab_variants.sh "nospec" 3 b1 $O/ab_r4f.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_model_small.py tests/test_gpu_full.py -x -q --timeout 300 \
  --timeout-method thread > $O/sw_test2.log 2>&1
