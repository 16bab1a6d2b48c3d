#!/bin/bash
# B = 8 decode (configs[3] per-GPU share) with the o_proj MFMA GEMV at 4 / 1 / 2 waves per workgroup,
# after the small-model and op parity tests.  usage (via gpurun): bash tools/b8_waves.sh
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/b8
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_model_small.py $R/tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/b8/tests.log 2>&1
for i in 1 2; do for w in 4 1 2; do
PGMI_MF_O_WAVES=$w timeout -k 10 300 python $R/bench.py --no-448 --no-cpu-baseline --prefill-iters 3 --steps 64 --nokv-tokens 2 > $R/gpurun_out/b8/b_$w.json 2> /dev/null
echo "waves $w $(python3 -c 'import sys,json; d=json.load(open(sys.argv[1])); print(d["value"], d["config4_images_per_gpu"]["ms_per_step"], d["config4_images_per_gpu"]["decode_tok_s"])' $R/gpurun_out/b8/b_$w.json)"
done; done
