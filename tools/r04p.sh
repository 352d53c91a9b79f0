#!/bin/bash
# round-4 GPU pass p (run on the box): large-path tests with the rows-phase chains split in
# two (4-wide instance), then its A/B against the final build (fin)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_big.py tests/test_gpu_configs.py tests/test_gpu_robust.py tests/test_gpu_constraints.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04p_test.log 2>&1
rc=$?; tail -3 gpurun_out/r04p_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 bash tools/ab_big_env.sh "C3:1024" "nlp-filter_amd/mhe/libmhe.so tools/libmhe_fin.so" 4 || exit $?
cp gpurun_out/ab_big_env.log gpurun_out/r04p_ab_big_rows_split.txt
