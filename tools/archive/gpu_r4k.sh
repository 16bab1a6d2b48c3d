#!/bin/bash
# Round-4: register-streamed MFMA GEMVs with the default cache policy (the new default) vs non-temporal
# (libpgmi_mfnt.so): batched parity tests, then same-box B = 8 and B = 4 bench pairs.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_batch.py tests/test_gpu_model_small.py tests/test_gpu_ops.py -x -q \
  --timeout 300 --timeout-method thread > $O/t_mf.log 2>&1
bash tools/ab_variants.sh "mfnt" 2 b8 $O/ab_r4k.txt
for i in 1 2; do
  for v in base mfnt; do
    if [ $v = base ]; then unset PGMI_LIB_PATH; else export PGMI_LIB_PATH=$R/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi/libpgmi_$v.so; fi
    timeout -k 10 300 python bench.py --batch 4 --steps 64 --warmup 8 --no-448 --no-extra --no-api --no-cpu-baseline \
      --prefill-iters 3 > $O/b4.log 2>&1
    echo "b4 $v $(tail -n 1 $O/b4.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab_r4k.txt
  done
done
