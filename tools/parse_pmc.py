"""Summarise the rocprofv3 passes of tools/profile_round.sh for the k_gn kernel.

HBM traffic per launch = 2 * FETCH_SIZE + WRITE_SIZE (KB -> bytes):
MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are L2 memory-side request
counters in KB; on gfx950 FETCH_SIZE reports 1/2 of a wide coalesced stream,
so it is doubled (other access widths are uncalibrated -- stated in the note).
Writes profiles/pmc_summary.json (read by bench.py for roofline.traffic, stamped
with the sha256 of the libmhe.so that was profiled) and
copies the per-kernel stats CSV to profiles/<tag>_kernel_stats.csv."""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nlp-filter_amd"))
from mhe._lib import lib_digest  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
out = os.path.join(ROOT, "gpurun_out")


def rows(pass_name):
    fs = glob.glob(os.path.join(out, f"prof_{tag}_{pass_name}", "**", "*counter_collection.csv"), recursive=True)
    res = []
    for f in fs:
        res += list(csv.DictReader(open(f)))
    return res


def per_dispatch(pass_name, counter, how="sum"):
    """Per-dispatch value of `counter`: summed over its instances, or their max
    (GRBM_GUI_ACTIVE is reported once per XCD; the derived MfmaUtil uses the max)."""
    vals = {}
    for r in rows(pass_name):
        if "k_gn<mhe::DynVanDerPol" not in r.get("Kernel_Name", "") or r.get("Counter_Name") != counter:
            continue
        d, v = r["Dispatch_Id"], float(r["Counter_Value"])
        vals[d] = (vals.get(d, 0.0) + v) if how == "sum" else max(vals.get(d, 0.0), v)
    return list(vals.values())


def mean(v):
    return sum(v) / len(v) if v else None


fetch = mean(per_dispatch("fetch", "FETCH_SIZE"))
write = mean(per_dispatch("write", "WRITE_SIZE"))
mops = mean(per_dispatch("sq", "SQ_INSTS_VALU_MFMA_MOPS_F64"))
busy = mean(per_dispatch("sq", "SQ_VALU_MFMA_BUSY_CYCLES"))
gui = mean(per_dispatch("sq", "GRBM_GUI_ACTIVE", how="max"))
summary = {
    "tag": tag, "kernel_sig": "k_gn<DynVanDerPol", "batch": 1024, "iters": 10,
    # the build these counters measured: bench.py attaches them only to a run of the same libmhe.so
    "lib_sha": lib_digest(),
    "fetch_size_kb": fetch, "write_size_kb": write,
    "hbm_bytes_per_launch": None if fetch is None or write is None else (2.0 * fetch + write) * 1024.0,
    "mfma_f64_flops_per_launch": None if mops is None else mops * 512.0,
    "mfma_busy_cycles": busy, "grbm_gui_active": gui,
    # MfmaUtil = SQ_VALU_MFMA_BUSY_CYCLES (all SIMDs) / (GUI-active cycles of one XCD * 1024 SIMDs);
    # rocprofv3 reports GRBM_GUI_ACTIVE summed over the 8 XCDs (MI355X_MICROARCH.md DVFS note)
    "mfma_util": None if busy is None or not gui else busy / (gui / 8.0 * 1024.0),
    "note": "2*FETCH_SIZE + WRITE_SIZE (KB), gfx950 FETCH_SIZE halving corrected; 8-B scattered reads are "
            "uncalibrated (MI355X_MICROARCH.md §HBM); Infinity-Cache hits are counted",
}
# the kernel's launch durations from the trace pass, split into the bench's warm-up launches
# and its timed launches: bench.py's kernel_ms (HIP events around the timed launches) and
# the rocprof average over those same launches are one basis
durs = []
for f in glob.glob(os.path.join(out, f"prof_{tag}_trace", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_gn<mhe::DynVanDerPol" in r.get("Kernel_Name", "") and "MeasFullState" in r["Kernel_Name"]:
            durs.append((int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6))
durs = [d for _, d in sorted(durs)]
warm = int(os.environ.get("PROF_WARMUP", "2"))
if durs:
    summary["trace_launches"] = len(durs)
    summary["trace_ms_all_launches"] = sum(durs) / len(durs)
    timed = durs[warm:] if len(durs) > warm else durs
    summary["trace_ms_timed_launches"] = sum(timed) / len(timed)
    summary["trace_ms_first_launch"] = durs[0]
os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
with open(os.path.join(ROOT, "profiles", "pmc_summary.json"), "w") as f:
    json.dump(summary, f, indent=1)
for st in glob.glob(os.path.join(out, f"prof_{tag}_trace", "**", "*kernel_stats.csv"), recursive=True):
    shutil.copy(st, os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
print(json.dumps(summary))
