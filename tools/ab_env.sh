#!/bin/bash
# Same-box A/B of one environment knob on the decode bench: alternating short bench.py runs with
# and without the assignment.  usage (via gpurun): bash tools/ab_env.sh "<VAR=value ...>" [rounds] [448]
# (a third argument "448" adds the 448 px prefill to every run and prints its time too)
set -e
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/abenv
for i in $(seq 1 ${2:-3}); do
  for v in base knob; do
    if [ $v = knob ]; then E="$1"; else E=""; fi
    if [ "$3" = 448 ]; then X=""; else X="--no-448"; fi
    env $E timeout -k 10 300 python $GRAFT_REPO_ROOT/bench.py $X --no-extra --no-api --no-cpu-baseline --prefill-iters 3 \
      > $GRAFT_REPO_ROOT/gpurun_out/abenv/b.log 2>&1
    echo "$v $(tail -n 1 $GRAFT_REPO_ROOT/gpurun_out/abenv/b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["prefill_ms"], (d.get("prefill_448") or {}).get("prefill_ms", ""))')"
  done
done
