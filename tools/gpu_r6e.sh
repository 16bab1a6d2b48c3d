#!/bin/bash
# Round 6: the ping-pong GEMM (k_gemm_wp, cfgs 41-44) and the 32-deep-slot ring (k_gemm_h, cfgs 45-50) against
# k_gemm_w on the M = 288 prefill shapes, cold isolated and in situ; then tools/gpu_r6d.sh (diagnostic builds)
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6e
mkdir -p $OUT
cd $R
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/ops.log 2>&1
echo ops done
timeout -k 10 300 python -u tools/gemm_sweep.py t_gateup --cold --all --cfgs 31,41,43,45,48 --splits 1 > $OUT/iso_gateup.txt 2>&1
echo iso gateup done
timeout -k 10 300 python -u tools/gemm_sweep.py t_down t_o --cold --all --cfgs 30,34,41,42,44,46,47,48 --splits 4,8,16 > $OUT/iso_down.txt 2>&1
echo iso down done
timeout -k 10 300 python -u tools/gemm_sweep.py v_fc1 v_fc2 v_qkv v_out --cold --all --cfgs 25,28,47,49,50 --splits 1,2,4,8 > $OUT/iso_vision.txt 2>&1
echo iso vision done
timeout -k 10 400 python -u tools/probes/plan_sweep.py --target lm --shapes gateup,down,o --cfgs 31,34,41,44,45,46,47,48 \
    --splits 4,8,16 --rel-tol 5e-2 > $OUT/insitu.txt 2>&1
echo insitu done
