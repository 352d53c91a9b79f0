#!/bin/bash
# round-4 GPU pass h (run on the box): rows-below prefetch A/B on the large path
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 500 bash tools/ab_big_env.sh "C3:1024 C4:256" "nlp-filter_amd/mhe/libmhe.so tools/libmhe_rowspf.so" 3 || exit $?
cp gpurun_out/ab_big_env.log gpurun_out/r04h_ab_big_rowspf.txt
