#!/bin/bash
# Large-system path profile (run on the GPU box): per-kernel stats and HBM bytes
#   tools/prof_big.sh <C3|C4|C5> <B> <tag>   -> gpurun_out/pbig_<tag>_{trace,fetch,write}/
set -e
CFG=$1; B=$2; TAG=$3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R="python tools/bench_big.py $CFG $B 2"
timeout -k 10 300 $R > gpurun_out/pbig_${TAG}.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pbig_${TAG}_trace -o run -- $R > gpurun_out/pbig_${TAG}_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pbig_${TAG}_fetch -o run -- $R > gpurun_out/pbig_${TAG}_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pbig_${TAG}_write -o run -- $R > gpurun_out/pbig_${TAG}_write.log 2>&1
python - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
for p in ("fetch", "write"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"gpurun_out/pbig_{tag}_{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void mhe::", "")
            acc[k][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for k, d in acc.items():
        v = list(d.values())
        print(f"{p:5s} {k:28s} dispatches {len(v):3d} mean KB {sum(v)/len(v):14.1f}")
PY
