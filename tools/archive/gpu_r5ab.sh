#!/bin/bash
# Round 5 first GPU call: the parity tests and the bench line (gpu_r5a.sh), then the prefill GEMM hot / cold
# plan sweeps (gpu_r5b.sh).
set -e
bash $GRAFT_REPO_ROOT/tools/archive/gpu_r5a.sh
bash $GRAFT_REPO_ROOT/tools/archive/gpu_r5b.sh
