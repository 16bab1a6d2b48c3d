#!/bin/bash
# B = 8 decode (configs[3] per-GPU share): MLP on the MFMA GEMVs vs on the prefill GEMMs
# (PGMI_DEC_MLP_GEMM=8), parity tests with the GEMM form first.  usage (via gpurun): bash tools/b8_mlp.sh
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/b8m
PGMI_DEC_MLP_GEMM=3 timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_model_small.py -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/b8m/tests.log 2>&1
for i in 1 2; do for m in 0 8; do
PGMI_DEC_MLP_GEMM=$m timeout -k 10 300 python $R/bench.py --no-448 --no-cpu-baseline --prefill-iters 3 --steps 64 --nokv-tokens 2 > $R/gpurun_out/b8m/b_$m.json 2> /dev/null
echo "mlp_gemm $m $(python3 -c 'import sys,json; d=json.load(open(sys.argv[1])); print(d["value"], d["config4_images_per_gpu"]["ms_per_step"], d["config4_images_per_gpu"]["decode_tok_s"])' $R/gpurun_out/b8m/b_$m.json)"
done; done
