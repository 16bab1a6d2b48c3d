#!/bin/bash
# Round 6: the round's defaults (M = 288 gate|up on R288w, down on W288n split 8, Gemma 224 attention with 2
# compute waves) -- every -m gpu test with parity records, smoke, the bench line; then the diagnostic builds
# (built before the probe kernels were removed: R288w is cfg 52 there) on W288n against R288w
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6j
mkdir -p $OUT
cd $R
PGMI_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 \
    --timeout-method thread > $OUT/tests.log 2>&1
echo tests done
timeout -k 10 300 python3 -u -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > $OUT/smoke.log 2>&1
echo smoke done
timeout -k 10 500 python3 -u $R/bench.py --steps 20 > $OUT/bench.json 2> $OUT/bench.err
echo bench done
P=$R/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi
for v in diag1 diag2 diag3; do
  PGMI_LIB_PATH=$P/libpgmi_$v.so timeout -k 10 200 python -u tools/gemm_sweep.py t_gateup --cold --all --iters 40 \
      --cfgs 31,52 --splits 1 > $OUT/iso_$v.txt 2>&1
  echo $v done
done
