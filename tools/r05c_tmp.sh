cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05x
MHE_LIB=ab/libmhe_ts1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_big.py tests/test_gpu_big_parity.py > gpurun_out/${T}_bigtests.txt 2>&1 || { tail -30 gpurun_out/${T}_bigtests.txt; exit 1; }
tail -2 gpurun_out/${T}_bigtests.txt
timeout -k 10 1100 bash tools/ab_big.sh "nlp-filter_amd/mhe/libmhe.so ab/libmhe_ts1.so" "C3:1024 C4:256 C5:256" 2 > /dev/null 2>&1; cp gpurun_out/ab_big.log gpurun_out/${T}_ab_big.txt
cat gpurun_out/${T}_ab_big.txt
