#!/bin/bash
# Large-system path timing for a set of libraries (run on the GPU box):
#   tools/big_ab.sh "<libA.so> <libB.so> ..."   -> gpurun_out/big_ab.log
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/big_ab.log
: > $O
for L in $1; do
  for c in "C3 1024" "C4 256" "C5 1024"; do
    MHE_LIB=$L timeout -k 10 300 python tools/bench_big.py $c 2 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$L', d['config'], d['B'], round(d['ms_per_iter'],2), 'ms/iter', round(d['frac_fp64_peak'],3))" >> $O || exit 1
  done
done
