#!/bin/bash
# round-4 GPU pass n (run on the box): large-path tests with the double-buffered half-slab
# staging of the 8-wide left-looking update, then its A/B against HEAD (asm1)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_big.py tests/test_gpu_configs.py tests/test_gpu_robust.py tests/test_gpu_constraints.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04n_test.log 2>&1
rc=$?; tail -3 gpurun_out/r04n_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 bash tools/ab_big_env.sh "C4:256 C5:256" "nlp-filter_amd/mhe/libmhe.so tools/libmhe_asm1.so" 2 || exit $?
cp gpurun_out/ab_big_env.log gpurun_out/r04n_ab_big_dbuf.txt
