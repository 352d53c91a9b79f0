#!/bin/bash
# Instruction mix and MFMA busy of the large-system kernels (run on the GPU box):
#   tools/sq_big.sh <C3|C4> <B> <tag>   -> gpurun_out/sqbig_<tag>_{1,2}/, summary on stdout
# Separate --pmc passes (each within the per-block counter limits), --kernel-trace none.
set -e
CFG=$1; B=$2; TAG=$3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R="python tools/bench_big.py $CFG $B 1"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/sqbig_${TAG}_$i -o run -- $R > gpurun_out/sqbig_${TAG}_$i.log 2>&1
done
python - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
# per kernel: per dispatch sums (GRBM_GUI_ACTIVE: max over instances = one XCD's active cycles x 8 reported)
acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for f in glob.glob(f"gpurun_out/sqbig_{tag}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("<")[0].replace("void mhe::", "").strip()
        if not k.startswith("k_big"):
            continue
        c, d, v = r["Counter_Name"], r["Dispatch_Id"], float(r["Counter_Value"])
        if c == "GRBM_GUI_ACTIVE":
            acc[k][d][c] = max(acc[k][d][c], v)
        else:
            acc[k][d][c] += v
for k, ds in sorted(acc.items()):
    tot = collections.defaultdict(float)
    for d in ds.values():
        for c, v in d.items():
            tot[c] += v
    nd = len(ds)
    waves = tot.get("SQ_WAVES", 0.0) or 1.0
    line = {c: v / nd for c, v in tot.items()}
    per_wave = {c.replace("SQ_INSTS_", ""): round(tot[c] / waves, 1) for c in tot if c.startswith("SQ_INSTS_")}
    util = None
    if tot.get("GRBM_GUI_ACTIVE"):
        util = tot["SQ_VALU_MFMA_BUSY_CYCLES"] / (tot["GRBM_GUI_ACTIVE"] / 8.0 * 1024.0)
    print(f"{k:18s} dispatches {nd:3d} waves/dispatch {waves / nd:10.0f} per-wave {per_wave} "
          f"mfma_busy {util if util is None else round(util, 3)}")
PY
