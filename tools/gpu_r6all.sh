#!/bin/bash
# round 6: the whole -m gpu suite on the final sources, then smoke()
set -o pipefail
mkdir -p gpurun_out/r6all
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r6all/tests.log 2>&1 && echo tests done && \
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6all/smoke.log 2>&1 && \
echo smoke done
