#!/bin/bash
# round-4 GPU pass g (run on the box): suite, then the backward-solve A/B on the large path
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04g_gputest.log 2>&1
rc=$?; tail -3 gpurun_out/r04g_gputest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 bash tools/ab_big_env.sh "C3:1024 C4:256" "nlp-filter_amd/mhe/libmhe.so tools/libmhe_bwd0.so" 3 || exit $?
cp gpurun_out/ab_big_env.log gpurun_out/r04g_ab_big_bwd.txt
