#!/bin/bash
# Large-path A/B over library variants and env settings, alternating (run on the GPU box):
#   tools/ab_big_env.sh "<CFG:B> ..." "<lib.so>[,ENV=V] ..." [rounds]  -> gpurun_out/ab_big_env.log
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_big_env.log
: > $O
for i in $(seq ${3:-2}); do
  for CB in $1; do
    for LE in $2; do
      L=${LE%%,*}; E=""; [[ $LE == *,* ]] && E=${LE#*,}
      v=$(env MHE_LIB=$L $E timeout -k 10 300 python tools/bench_big.py ${CB%:*} ${CB#*:} 2 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_iter'], d['frac_fp64_peak'])") || exit 1
      echo "$CB $LE $v" | tee -a $O
    done
  done
done
