#!/bin/bash
# Same-box A/B of environment settings on the B = 8 decode step (configs[3] per-GPU share):
# alternating short bench.py runs, one per setting ("" = defaults), printing the B = 1 value and
# the B = 8 step.  usage (via gpurun): bash tools/b8_env.sh [rounds] "<VAR=v ...>" "<VAR=v ...>" ...
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/b8env
N=$1; shift
for i in $(seq 1 $N); do
  for E in "" "$@"; do
    env $E timeout -k 10 300 python $R/bench.py --no-448 --no-api --no-cpu-baseline --prefill-iters 3 --steps 32 \
      --nokv-tokens 2 > $R/gpurun_out/b8env/b.json 2> /dev/null
    echo "[$E] $(python3 -c 'import sys,json; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d["config4_images_per_gpu"]; print(d["value"], c["ms_per_step"], c["decode_tok_s"])' $R/gpurun_out/b8env/b.json)"
  done
done
