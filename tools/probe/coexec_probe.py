"""f64 MFMA vs VALU co-issue on one SIMD (tools only; see coexec_probe.hip)."""
import ctypes, os, torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libcoexec_probe.so"))
out = torch.zeros(512, dtype=torch.float64, device="cuda"); cyc = torch.zeros(8, dtype=torch.int64, device="cuda")
iters = 2000
for mode, name in ((1, "MFMA waves alone"), (2, "f64 FMA waves alone"), (3, "MFMA + f64 FMA"),
                   (4, "int32 waves alone"), (5, "MFMA + int32"), (18, "f64 FMA, 2 waves/SIMD"),
                   (11, "MFMA + f64 FMA prio 3"), (35, "1-chain MFMA + f64 FMA"), (33, "1-chain MFMA alone")):
    for _ in range(2):
        lib.run(ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(cyc.data_ptr()), mode, iters)
    c = cyc.cpu().tolist()
    print(f"{name:24s} MFMA waves {sum(c[:4]) / 4 / (iters * 8):7.1f} cyc/MFMA   "
          f"VALU waves {sum(c[4:]) / 4 / (iters * 16 * 8):6.2f} cyc/op   (raw {c})")
