#!/bin/bash
# round-4 GPU pass e (run on the box): suite, then assemble A/B (grouped LDS-staged vs coalesced)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04e_gputest.log 2>&1
rc=$?; tail -3 gpurun_out/r04e_gputest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 bash tools/ab_big_env.sh "C3:1024 C4:256" "nlp-filter_amd/mhe/libmhe.so tools/libmhe_asmcoal.so" 2 || exit $?
cp gpurun_out/ab_big_env.log gpurun_out/r04e_ab_big.txt
