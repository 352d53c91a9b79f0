cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MHE_BIG_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/psplit_trace -o run -- python tools/bench_big.py C3 1024 2 > gpurun_out/psplit.log 2>&1 || exit $?
MHE_BIG_SPLIT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pbase_trace -o run -- python tools/bench_big.py C3 1024 2 > gpurun_out/pbase.log 2>&1
