#!/bin/bash
# round-4 GPU pass k (run on the box): EKF tests, then the lane-kernel occupancy A/B
# (product: S upper triangle for every n + per-model waves-per-SIMD bound; ekf0: before)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ekf.py tests/test_ekf_autocar.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04k_ekftest.log 2>&1
rc=$?; tail -3 gpurun_out/r04k_ekftest.log; [ $rc -ne 0 ] && exit $rc
O=gpurun_out/r04k_ab_ekf.txt; : > $O
for i in 1 2; do
  for L in nlp-filter_amd/mhe/libmhe.so tools/libmhe_ekf0.so; do
    v=$(NO_CPU=1 MHE_LIB=$L timeout -k 10 200 python tools/bench_ekf.py 262144 10 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_launch'], d['value'], d['roofline']['frac'])") || exit 1
    echo "gnss_n5_B262144 $L $v" | tee -a $O
    v=$(NO_CPU=1 MHE_LIB=$L timeout -k 10 200 python tools/bench_ekf_autocar.py 131072 5 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['kernel_ms'], d['filter_steps_per_s'])") || exit 1
    echo "autocar_n9_B131072 $L $v" | tee -a $O
  done
done
