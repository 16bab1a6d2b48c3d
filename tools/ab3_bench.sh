#!/bin/bash
# Same-box comparison of libpgmi_base.so, libpgmi.so and libpgmi.so under an extra env setting
# (e.g. PGMI_LM_FOLD=0): alternating short bench.py decode runs.
# usage (via gpurun): bash tools/ab3_bench.sh "<ENV=VAL>" [rounds]
set -e
R=$GRAFT_REPO_ROOT
B=$R/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi/libpgmi_base.so
mkdir -p $R/gpurun_out/ab
for i in $(seq 1 ${2:-2}); do
  for v in base new env; do
    unset PGMI_LIB_PATH
    EXTRA=""
    if [ $v = base ]; then export PGMI_LIB_PATH=$B; fi
    if [ $v = env ]; then EXTRA="$1"; fi
    env $EXTRA timeout -k 10 300 python $R/bench.py --no-448 --no-extra --no-cpu-baseline --prefill-iters 3 \
      > $R/gpurun_out/ab/b.log 2>&1
    echo "$v $(tail -n 1 $R/gpurun_out/ab/b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["prefill_ms"])')"
  done
done
