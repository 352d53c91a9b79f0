#!/bin/bash
# A/B of libmhe builds at several per-GPU batches (run on the GPU box):
#   tools/gpu_ab.sh <tag> "<libA> <libB> ..." "<batches>" [rounds]  -> gpurun_out/<tag>_ab_B<batch>.txt
TAG=$1; LIBS=$2; BATCHES=${3:-"1024"}; R=${4:-3}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for B in $BATCHES; do
  bash tools/ab.sh "$LIBS" $R $B ${TAG}_ab_B$B.txt || exit $?
  tail -3 gpurun_out/${TAG}_ab_B$B.txt
done
