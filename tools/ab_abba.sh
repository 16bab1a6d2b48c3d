#!/bin/bash
# Same-box A/B of two library builds in balanced order (A B B A per round, so a drift over the run or a
# first-of-pair effect cancels): tools/probes/decode_only.py under PGMI_LIB_PATH for each.
# usage (via gpurun): bash tools/ab_abba.sh LIB_A LIB_B [rounds] [batch]
set -o pipefail
A=$1; B=$2; R=${3:-3}; NB=${4:-1}
for i in $(seq 1 $R); do
  for L in $A $B $B $A; do
    PGMI_LIB_PATH=$L timeout -k 10 240 python -u $GRAFT_REPO_ROOT/tools/probes/decode_only.py --batch $NB 2>&1 \
      | grep median || exit 1
  done
done
