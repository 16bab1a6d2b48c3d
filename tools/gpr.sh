#!/bin/bash
# Local wrapper around gpurun: retries only while the pool reports no free slot / box
# (status "transient": nothing ran, nothing charged).  usage: tools/gpr.sh <log> <timeout> <command>
LOG=$1; TO=$2; shift 2
for i in $(seq 1 25); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('/root/repo/gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  if [ "$st" = "transient" ]; then sleep 90; continue; fi
  break
done
echo "rc=$rc status=$st attempts=$i" >> $LOG
