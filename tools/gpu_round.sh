#!/bin/bash
# One GPU-box pass (run on the box): GPU tests, C2 bench, C2 profiles, C3/C4 large-path lines.
#   tools/gpu_round.sh <tag>   -> gpurun_out/<tag>_{gputest.log,bench.log,big_C3.json,big_C4.json}, prof_<tag>_*
# A failing test (pytest exit 1) does not stop the pass; any other exit status of a GPU
# step (crash, abort, time limit) ends it there.
TAG=${1:-r03}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
bash tools/profile_round.sh ${TAG} || exit $?
timeout -k 10 200 python tools/bench_big.py C3 4096 3 > gpurun_out/${TAG}_big_C3.json 2>&1 || exit $?
timeout -k 10 200 python tools/bench_big.py C4 1024 2 > gpurun_out/${TAG}_big_C4.json 2>&1 || exit $?
exit $rc
