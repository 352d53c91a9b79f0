#!/bin/bash
# round-4 GPU pass q (run on the box): the C2 parity tests (incl. small-batch vs full-occupancy instance)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04q_parity.log 2>&1
rc=$?; tail -3 gpurun_out/r04q_parity.log; exit $rc
