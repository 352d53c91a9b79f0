cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05b_parity.log 2>&1
rc=$?; tail -3 gpurun_out/r05b_parity.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh r05b "ab/libmhe_base.so ab/libmhe_sb.so" "128 256 1024" 3
