"""Instruction mix per GN phase group of the fused kernel (tools only; GPU + PMC).

    rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_F64 \
        -- python tools/valu_split.py
then  python tools/valu_split.py --parse <counter_collection.csv>

Launches (C2, B = 1024) the same k_gn instantiation in three modes:
  MODE_ASSEMBLE  residual + gradient + tile build of one iterate (no factorization)
  MODE_LINSOLVE  factorization + forward/backward solve of a given H, g
  MODE_SOLVE     1 and 3 full GN iterations (difference = per-iteration cost)
"""
import csv
import os
import sys
from collections import defaultdict

if len(sys.argv) > 2 and sys.argv[1] == "--parse":
    rows = list(csv.DictReader(open(sys.argv[2])))
    by = defaultdict(dict)
    for r in rows:
        if "k_gn" not in r["Kernel_Name"]:
            continue
        by[int(r["Dispatch_Id"])][r["Counter_Name"]] = by[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for d in sorted(by):
        c = by[d]
        print(d, {k: f"{v / 1024 / 8:.0f}" for k, v in sorted(c.items())}, "(per wave)")
    sys.exit(0)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nlp-filter_amd"))
import torch  # noqa: E402
from mhe import configs, solver  # noqa: E402

w = configs.make_c2(B=1024)
s = solver.from_workload(w)
H, g, _ = s.assemble(w.X_init, w.U, w.Y)           # dispatch: assemble
torch.cuda.synchronize()
s.chol_solve(H, g)                                  # dispatch: linsolve
torch.cuda.synchronize()
s.solve(w.X_init, w.U, w.Y, max_iter=1, tol=0.0)    # dispatch: 1 iteration
torch.cuda.synchronize()
s.solve(w.X_init, w.U, w.Y, max_iter=3, tol=0.0)    # dispatch: 3 iterations
torch.cuda.synchronize()
print("done")
