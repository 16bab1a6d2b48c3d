#!/bin/bash
# Iteration run on the GPU box: GPU parity tests (optionally -k), the default bench line, and
# (optional 3rd arg "list") the rocprofv3 counter list.  usage: bash tools/gpu_iter.sh <tag> [k-expr] [list]
set -e
TAG=${1:-iter}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$2" ] && [ "$2" != "all" ]; then K="-k $2"; else K=""; fi
timeout -k 10 700 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread $K > $OUT/tests.log 2>&1
echo tests done
timeout -k 10 400 python3 -u $R/bench.py > $OUT/bench.json 2> $OUT/bench.err
echo bench done
if [ "$3" = "list" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
fi
echo done
