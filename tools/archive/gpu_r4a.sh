#!/bin/bash
# Round-4 GPU check: parity tests of the touched areas (per-step rel-L2 records to
# gpurun_out/parity_tests.jsonl), smoke, the default bench line, then a same-box A/B of the batched
# (B = 8) decode step: the attention combine folded into the attention launch (PGMI_FUSED_COMB=1) or not.
# usage (via gpurun): bash tools/archive/gpu_r4a.sh [tests]
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
export PGMI_PARITY_LOG=$O/parity_tests.jsonl
T=${1:-"tests/test_gpu_modules.py tests/test_gpu_api.py tests/test_gpu_model_small.py tests/test_gpu_ablation.py tests/test_gpu_full.py tests/test_gpu_full_batch.py"}
cd $R
timeout -k 10 900 python -u -m pytest $T -x -v --timeout 300 --timeout-method thread > $O/t1.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > $O/bench1.log 2>&1
for i in 1 2; do
  for v in 0 1; do
    PGMI_FUSED_COMB=$v timeout -k 10 300 python bench.py --batch 8 --steps 64 --warmup 8 --no-448 --no-extra --no-api \
      --no-cpu-baseline --prefill-iters 3 > $O/b8.log 2>&1
    echo "comb=$v $(tail -n 1 $O/b8.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["prefill_ms"])')" >> $O/b8ab.txt
  done
done
