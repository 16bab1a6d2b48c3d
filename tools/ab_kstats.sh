#!/bin/bash
# Same-box A/B of two builds of libpgmi at kernel level: rocprofv3 kernel-trace stats of a short
# decode-only bench.py run with each (base = pgmi/libpgmi_base.so, new = pgmi/libpgmi.so).
# usage (via gpurun): bash tools/ab_kstats.sh <tag> [bench.py args; default: decode + 224 prefill only]
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
shift
BENCH_ARGS=${@:-"--no-448 --no-extra --no-api --no-cpu-baseline --prefill-iters 3 --steps 64"}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in base new; do
  if [ $v = base ]; then export PGMI_LIB_PATH=$R/multimodal-financial-analysis-tool-using-paligemma_amd/pgmi/libpgmi_base.so; else unset PGMI_LIB_PATH; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o run -- \
      python3 $R/bench.py ${BENCH_ARGS} > $OUT/$v.log 2>&1
  echo "$v done"
done
