#!/bin/bash
# round-4 closing profile pass (run on the box): C2 kernel trace + PMC passes (stamped
# pmc_summary.json), the large-path bench lines at the configured batches, kernel stats
# and HBM bytes of C3 / C4, and the instruction mix of the large-path kernels at C3.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 bash tools/profile_round.sh r04 > gpurun_out/r04_profile_round.log 2>&1 || exit $?
for cb in "C3 4096 3" "C4 1024 2" "C5 2048 2"; do
  timeout -k 10 400 python tools/bench_big.py $cb >> gpurun_out/r04_big_path.jsonl 2>/dev/null || exit $?
  tail -1 gpurun_out/r04_big_path.jsonl
done
timeout -k 10 400 bash tools/prof_big.sh C3 1024 r04_C3 > gpurun_out/r04_prof_big_C3.txt 2>&1 || exit $?
timeout -k 10 400 bash tools/prof_big.sh C4 256 r04_C4 > gpurun_out/r04_prof_big_C4.txt 2>&1 || exit $?
timeout -k 10 300 bash tools/sq_big.sh C3 1024 r04_C3 > gpurun_out/r04_sq_big_C3.txt 2>&1 || exit $?
cat gpurun_out/r04_prof_big_C3.txt gpurun_out/r04_sq_big_C3.txt
