#!/bin/bash
# Same-box A/B of library builds: pgmi/libpgmi.so ("base") against pgmi/libpgmi_<v>.so for each v,
# alternating short bench.py runs at batch 1 (mode b1) or 8 (mode b8).
# usage (via gpurun): bash tools/ab_variants.sh "v1 v2" [rounds] [b1|b8] [out-file]
set -e
R=$GRAFT_REPO_ROOT
P=$R/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi
O=${4:-$R/gpurun_out/ab_variants.txt}
MODE=${3:-b1}
for i in $(seq 1 ${2:-2}); do
  for v in base $1; do
    if [ $v = base ]; then unset PGMI_LIB_PATH; else export PGMI_LIB_PATH=$P/libpgmi_$v.so; fi
    if [ $MODE = b8 ]; then X="--batch 8 --steps 64 --warmup 8"; else X="--steps 256 --warmup 16"; fi
    timeout -k 10 300 python $R/bench.py $X --no-448 --no-extra --no-api --no-cpu-baseline --prefill-iters 3 \
      > $R/gpurun_out/abv.log 2>&1
    echo "$MODE $v $(tail -n 1 $R/gpurun_out/abv.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["prefill_ms"])')" >> $O
  done
done
