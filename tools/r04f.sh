#!/bin/bash
# round-4 GPU pass f (run on the box): knock-out timing of the k_big_chol phases (X frozen)
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 700 bash tools/ab_big_env.sh "C3:1024 C4:256" "tools/libmhe_kob64.so tools/libmhe_kob1.so tools/libmhe_kob2.so tools/libmhe_kob4.so tools/libmhe_kob16.so tools/libmhe_kob32.so" 1 || exit $?
cp gpurun_out/ab_big_env.log gpurun_out/r04f_ko_big.txt
