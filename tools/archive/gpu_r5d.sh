#!/bin/bash
# Round 5: k_gemm_w with exact LDS waits (kk=1 fragment reads under the kk=0 MFMAs) against the previous build
# (libpgmi_base.so) on the shapes its plans serve; then the GPU parity tests and the default bench line.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5d
mkdir -p $OUT
P=$R/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi
for rep in 1 2; do
  for lib in libpgmi_base libpgmi; do
    echo "== $lib rep $rep" >> $OUT/ab.txt
    PGMI_LIB_PATH=$P/$lib.so timeout -k 10 200 python3 -u $R/tools/gemm_sweep.py t_gateup t_qkv --cfgs 31,32 --splits 1 --all >> $OUT/ab.txt 2>&1
    PGMI_LIB_PATH=$P/$lib.so timeout -k 10 200 python3 -u $R/tools/gemm_sweep.py t_down t_o --cfgs 34,31 --splits 4,8 --all >> $OUT/ab.txt 2>&1
    PGMI_LIB_PATH=$P/$lib.so timeout -k 10 200 python3 -u $R/tools/gemm_sweep.py t448_qkv t448_o b8_t_o b8_v_fc2 b8_t_down --cfgs 34,31,30 --splits 1,2 --all >> $OUT/ab.txt 2>&1
  done
done
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
timeout -k 10 500 python3 -u $R/bench.py > $OUT/bench.json 2> $OUT/bench.err
echo done
