cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for B in 128 256 512; do
  timeout -k 10 300 python bench.py --global-batch $B --steps 20 --warmup 5 > gpurun_out/r05_bench_B$B.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r05_bench_B1024_nocpu.log 2>&1 || exit $?
for f in gpurun_out/r05_bench_B*.log; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], '%.4g' % d['value'], d['roofline']['kernel'], d['roofline'].get('traffic'))" $f; done
