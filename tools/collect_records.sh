#!/bin/bash
# Copy one tools/reproduce.sh run's outputs (gpurun_out/, tag $1) into profiles/ under the
# round name $2 (e.g. r06): the files DESIGN.md cites.
set -e
T=${1:?usage: tools/collect_records.sh <run tag> <round>}; R=${2:?round}
cd "$(dirname "$0")/.."
G=gpurun_out; P=profiles
cp $G/pmc_summary_$T.json $P/pmc_summary.json
cp $G/${T}_kernel_stats.csv $P/${R}_kernel_stats.csv
cp $G/${T}_bench.log $P/${R}_bench.log
cp $G/${T}_big_path.jsonl $P/${R}_big_path.jsonl
cp $G/${T}_prof_big_C3.txt $P/${R}_big_C3_hbm.txt
cp $G/${T}_prof_big_C4.txt $P/${R}_big_C4_hbm.txt
cp $G/pbig_${T}_C3_trace/run_kernel_stats.csv $P/${R}_big_C3_B1024_kernel_stats.csv
cp $G/pbig_${T}_C4_trace/run_kernel_stats.csv $P/${R}_big_C4_B256_kernel_stats.csv
cp $G/${T}_sq_big_C3.txt $P/${R}_sq_big_C3.txt
cp $G/${T}_gputest.log $P/${R}_gputest.log
cp $G/${T}_smoke.log $P/${R}_smoke.log
