"""Dependent-latency microbenchmarks (tools only): cycles per op in a 64-op chain."""
import ctypes, os, torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblat_probe.so"))
out = torch.zeros(64, dtype=torch.float64, device="cuda"); cyc = torch.zeros(1, dtype=torch.int64, device="cuda")
names = ["v_fma_f64", "v_rsq_f64 + add", "2 v_readlane + mul", "MFMA f64 16x16x4 (acc chain)", "MFMA -> A operand",
         "2 v_permlane16_swap + mul", "v_mul_f64", "v_rcp_f64 + add", "MFMA -> VALU mul -> MFMA"]
for w, nm in enumerate(names):
    for _ in range(3):
        lib.lat_run(w, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(cyc.data_ptr()))
    print(f"{nm:32s} {cyc.item() / 64:7.1f} cycles/op")
