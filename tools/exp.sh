#!/bin/bash
# Quick GPU experiment loop for the fused kernel (run on the GPU box):
# C2 parity tests, in-kernel phase stamps (1 and 2 workgroups per CU), bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/exp_${1:-x}.log
: > $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_robust.py -x -q --timeout 120 --timeout-method thread >> $O 2>&1 || { echo "TESTS FAILED" >> $O; exit 1; }
timeout -k 10 120 python tools/diag_phases.py 256 4 >> $O 2>&1 || exit 1
timeout -k 10 120 python tools/diag_phases.py 1024 4 >> $O 2>&1 || exit 1
timeout -k 10 120 python bench.py --no-cpu >> $O 2>&1 && timeout -k 10 120 python bench.py --no-cpu >> $O 2>&1 || exit 1
