#!/bin/bash
# Round-4 full GPU pass: every -m gpu test (per-step parity records to gpurun_out/parity_tests.jsonl),
# smoke, the default bench line, a same-box A/B of the batched (B = 8) attention combine fold, and the
# rocprofv3 kernel-trace stats of a short bench run (profiles/r04_kernel_stats.csv).
# usage (via gpurun): bash tools/archive/gpu_r4b.sh
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
export PGMI_PARITY_LOG=$O/parity_tests.jsonl
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_all.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > $O/bench1.log 2>&1
for i in 1 2; do
  for v in 0 1; do
    PGMI_FUSED_COMB=$v timeout -k 10 300 python bench.py --batch 8 --steps 64 --warmup 8 --no-448 --no-extra --no-api \
      --no-cpu-baseline --prefill-iters 3 > $O/b8.log 2>&1
    echo "comb=$v $(tail -n 1 $O/b8.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["prefill_ms"])')" >> $O/b8ab.txt
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r04/trace -o run -- \
    python3 $R/bench.py --steps 64 --warmup 8 --no-cpu-baseline --prefill-iters 5 > $O/prof_r04_bench.log 2>&1
echo done
