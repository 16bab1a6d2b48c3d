#!/bin/bash
# Same-box A/B of B = 8 decode across library builds (pgmi/libpgmi.so and pgmi/libpgmi_<v>.so):
# bench.py --batch 8 decode ms/step, alternating.  usage (via gpurun): bash tools/b8_ab.sh "v1 v2" [rounds]
set -e
P=$GRAFT_REPO_ROOT/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/b8ab
for i in $(seq 1 ${2:-1}); do
  for v in base $1; do
    if [ $v = base ]; then unset PGMI_LIB_PATH; else export PGMI_LIB_PATH=$P/libpgmi_$v.so; fi
    timeout -k 10 300 python $GRAFT_REPO_ROOT/bench.py --batch 8 --steps 64 --warmup 8 --no-448 --no-extra --no-api \
      --no-cpu-baseline --prefill-iters 3 > $GRAFT_REPO_ROOT/gpurun_out/b8ab/b.log 2>&1
    echo "$v $(tail -n 1 $GRAFT_REPO_ROOT/gpurun_out/b8ab/b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["prefill_ms"])')"
  done
done
