#!/bin/bash
# round-4 GPU pass m (run on the box): large-path tests with the fused rows pass of the
# left-looking factorization, then its A/B against the unfused build (asm1 = HEAD)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_big.py tests/test_gpu_configs.py tests/test_gpu_robust.py tests/test_gpu_constraints.py tests/test_gpu_streams.py tests/test_gpu_autocar.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04m_test.log 2>&1
rc=$?; tail -5 gpurun_out/r04m_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 bash tools/ab_big_env.sh "C3:1024 C4:256" "nlp-filter_amd/mhe/libmhe.so tools/libmhe_asm1.so" 3 || exit $?
cp gpurun_out/ab_big_env.log gpurun_out/r04m_ab_big_fused.txt
