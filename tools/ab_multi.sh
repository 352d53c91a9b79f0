#!/bin/bash
# A/B over several batch sizes: tools/ab_multi.sh "<libs>" "<batches>" [rounds] -> gpurun_out/ab_B<batch>.log
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for B in $2; do
  timeout -k 10 400 bash tools/ab.sh "$1" ${3:-2} $B || exit 1
  cp gpurun_out/ab.log gpurun_out/ab_B$B.log
  grep mean gpurun_out/ab_B$B.log | sed "s/^/B=$B /"
done
