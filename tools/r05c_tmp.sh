cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05z
MHE_LIB=ab/libmhe_monof.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_big.py tests/test_gpu_big_parity.py > gpurun_out/${T}_bigtests.txt 2>&1 || { tail -30 gpurun_out/${T}_bigtests.txt; exit 1; }
tail -2 gpurun_out/${T}_bigtests.txt
timeout -k 10 1100 bash tools/ab_big.sh "nlp-filter_amd/mhe/libmhe.so ab/libmhe_monof.so" "C3:1024 C3:4096" 2 > /dev/null 2>&1; cp gpurun_out/ab_big.log gpurun_out/${T}_ab_big.txt
cat gpurun_out/${T}_ab_big.txt
MHE_LIB=ab/libmhe_monof.so timeout -k 10 400 bash tools/prof_big.sh C3 1024 ${T}_C3 > gpurun_out/${T}_prof_C3.txt 2>&1 || exit $?
grep -i "chol" gpurun_out/${T}_prof_C3.txt
