#!/bin/bash
# Kernel trace + separate PMC passes for the bench workload (run on the GPU box).
#   tools/profile_round.sh <tag>     -> gpurun_out/prof_<tag>_{trace,fetch,write,sq}/
set -e
TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --steps 10 --warmup 2 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_trace -o run -- $B > gpurun_out/prof_${TAG}_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_${TAG}_fetch -o run -- $B > gpurun_out/prof_${TAG}_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_${TAG}_write -o run -- $B > gpurun_out/prof_${TAG}_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --output-format csv -d gpurun_out/prof_${TAG}_sq -o run -- $B > gpurun_out/prof_${TAG}_sq.log 2>&1
python tools/parse_pmc.py "$TAG"
# profiles/ on the box is not copied back: hand the summary and stats over through gpurun_out/
cp profiles/pmc_summary.json "gpurun_out/pmc_summary_${TAG}.json"
cp "profiles/${TAG}_kernel_stats.csv" "gpurun_out/${TAG}_kernel_stats.csv"
