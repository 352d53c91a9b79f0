#!/bin/bash
# One GPU-box pass (run on the box): the GPU test suite, the default bench line, then
# optional A/B of libmhe builds:  tools/gpu_quick.sh <tag> ["<libA> <libB>" "<batches>"]
TAG=${1:-r04}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_gputest.log
if [ $rc -ne 0 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -c 600 gpurun_out/${TAG}_bench.log
if [ -n "$2" ]; then bash tools/gpu_ab.sh $TAG "$2" "$3" 3 || exit $?; fi
