#!/bin/bash
# A/B of the large-system path: tools/ab_big.sh "<libA.so> <libB.so>" "<CFG:B> ..." [rounds]
# -> gpurun_out/ab_big.log (ms per GN iteration from tools/bench_big.py, builds alternating)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_big.log
: > $O
for i in $(seq ${3:-2}); do
  for CB in $2; do
    for L in $1; do
      v=$(MHE_LIB=$L timeout -k 10 300 python tools/bench_big.py ${CB%:*} ${CB#*:} 2 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_iter'], d['frac_fp64_peak'])") || exit 1
      echo "$CB $L $v" | tee -a $O
    done
  done
done
