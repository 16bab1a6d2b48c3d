#!/bin/bash
# Same-box A/B of two builds of libpgmi (base = pgmi/libpgmi_base.so, new = pgmi/libpgmi.so):
# alternating short bench.py decode runs.  usage (via gpurun): bash tools/ab_bench.sh [rounds] [448]
# (a second argument "448" adds the 448 px prefill to every run and prints its time too)
set -e
B=$GRAFT_REPO_ROOT/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi/libpgmi_base.so
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/ab
for i in $(seq 1 ${1:-2}); do
  for v in base new; do
    if [ $v = base ]; then export PGMI_LIB_PATH=$B; else unset PGMI_LIB_PATH; fi
    if [ "$2" = 448 ]; then X=""; else X="--no-448"; fi
    timeout -k 10 300 python $GRAFT_REPO_ROOT/bench.py $X --no-extra --no-api --no-cpu-baseline --prefill-iters 3 \
      > $GRAFT_REPO_ROOT/gpurun_out/ab/b.log 2>&1
    echo "$v $(tail -n 1 $GRAFT_REPO_ROOT/gpurun_out/ab/b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["prefill_ms"], (d.get("prefill_448") or {}).get("prefill_ms", ""))')"
  done
done
