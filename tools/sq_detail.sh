#!/bin/bash
# Extra SQ counter passes (issue-level view of k_gn).  tools/sq_detail.sh <tag>
set -e
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --steps 3 --warmup 1 --no-cpu"
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_F64" \
           "SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/sq_${TAG}_$i -o run -- $B > gpurun_out/sq_${TAG}_$i.log 2>&1
done
python - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
tot = collections.defaultdict(float); n = collections.defaultdict(int)
for f in glob.glob(f"gpurun_out/sq_{tag}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_gn" not in r["Kernel_Name"]: continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
launches = max(1, max(n.values()) if n else 1)
for k in sorted(tot):
    print(f"{k:32s} {tot[k]:.4e}  dispatches-rows={n[k]}")
PY
