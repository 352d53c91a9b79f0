cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/r05d_diag.txt
for L in diag_sb; do for B in 128; do
  MHE_DIAG_LIB=ab/libmhe_$L.so timeout -k 10 120 python tools/diag_phases.py $B 4 >> gpurun_out/r05d_diag.txt 2>&1 || exit $?
done; done
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05d_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r05d_parity.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh r05d "ab/libmhe_base.so ab/libmhe_sb.so" "128 256" 3
cat gpurun_out/r05d_diag.txt
