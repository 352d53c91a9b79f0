#!/bin/bash
# k_big_chol (MHE_BIG_SPLIT=0) vs the split factorization (=1), alternating:
#   tools/ab_split.sh "<CFG:B> ..." [rounds]   -> gpurun_out/ab_split.log
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_split.log
: > $O
for i in $(seq ${2:-2}); do
  for CB in $1; do
    for S in 0 1; do
      v=$(MHE_BIG_SPLIT=$S timeout -k 10 300 python tools/bench_big.py ${CB%:*} ${CB#*:} 2 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_iter'], d['frac_fp64_peak'])") || exit 1
      echo "$CB split=$S $v" | tee -a $O
    done
  done
done
