#!/bin/bash
# How every number DESIGN.md quotes is produced (run on the GPU box through gpurun):
#   tools/reproduce.sh <tag> [suite] [close] [big]      (default: all three parts)
#     suite  pytest -m gpu, then __graft_entry__.smoke()
#     close  C2: kernel trace + separate PMC passes (tools/profile_round.sh ->
#            profiles/pmc_summary.json stamped with the profiled libmhe.so sha,
#            <tag>_kernel_stats.csv), then the default bench line, which attaches them
#     big    large-system path: bench lines at the configured batches (tools/bench_big.py
#            -> <tag>_big_path.jsonl), kernel stats + HBM bytes of C3 / C4
#            (tools/prof_big.sh), instruction mix at C3 (tools/sq_big.sh)
# Everything lands in gpurun_out/ (copied into profiles/ by hand afterwards).  Every GPU
# step has its own time limit and the first failure ends the script.
TAG=${1:?usage: tools/reproduce.sh <tag> [suite] [close] [big]}
shift
PARTS=${*:-suite close big}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
python -c "import sys; sys.path.insert(0, 'nlp-filter_amd'); from mhe import _lib; print('libmhe.so sha256[:16]', _lib.lib_digest())"
for part in $PARTS; do
  case $part in
  suite)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1
    rc=$?; tail -3 gpurun_out/${TAG}_gputest.log; [ $rc -ne 0 ] && exit $rc
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
    tail -1 gpurun_out/${TAG}_smoke.log ;;
  close)
    timeout -k 10 600 bash tools/profile_round.sh $TAG > gpurun_out/${TAG}_profile_round.log 2>&1 || exit $?
    tail -c 600 gpurun_out/${TAG}_profile_round.log
    timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
    tail -c 1500 gpurun_out/${TAG}_bench.log ;;
  big)
    for cb in "C3 4096 3" "C4 1024 2" "C5 2048 2"; do
      timeout -k 10 400 python tools/bench_big.py $cb >> gpurun_out/${TAG}_big_path.jsonl 2>/dev/null || exit $?
      tail -1 gpurun_out/${TAG}_big_path.jsonl
    done
    timeout -k 10 400 bash tools/prof_big.sh C3 1024 ${TAG}_C3 > gpurun_out/${TAG}_prof_big_C3.txt 2>&1 || exit $?
    timeout -k 10 400 bash tools/prof_big.sh C4 256 ${TAG}_C4 > gpurun_out/${TAG}_prof_big_C4.txt 2>&1 || exit $?
    timeout -k 10 300 bash tools/sq_big.sh C3 1024 ${TAG}_C3 > gpurun_out/${TAG}_sq_big_C3.txt 2>&1 || exit $?
    cat gpurun_out/${TAG}_prof_big_C3.txt gpurun_out/${TAG}_sq_big_C3.txt ;;
  *) echo "unknown part $part"; exit 2 ;;
  esac
done
