#!/bin/bash
# round-4 closing pass (run on the box): GPU suite, smoke, the C2 profile passes stamped to
# this build (pmc_summary.json), then the default bench line, which picks that summary up.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04z_gputest.log 2>&1
rc=$?; tail -3 gpurun_out/r04z_gputest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04z_smoke.log 2>&1 || exit $?
tail -2 gpurun_out/r04z_smoke.log
timeout -k 10 600 bash tools/profile_round.sh r04 > gpurun_out/r04z_profile_round.log 2>&1 || exit $?
tail -c 600 gpurun_out/r04z_profile_round.log
timeout -k 10 300 python bench.py > gpurun_out/r04z_bench.log 2>&1 || exit $?
tail -c 1500 gpurun_out/r04z_bench.log
