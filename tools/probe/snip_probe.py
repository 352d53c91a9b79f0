"""Cycle costs of code shapes (tools only).  Empty-rep overhead subtracted is NOT done: compare rows."""
import ctypes, os, torch
here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "libsnip_probe.so"))
names = ["T: 1 tile (4 dep MFMA + 4 ds_write)", "T: 3 tiles", "U: 10 tiles naive", "U: 10 tiles 2-interleaved",
         "40 MFMA on 10 accs", "40 dependent MFMA", "LDS store->load round trip", "16 readlane-pair + fma chain"]
for v, nm in enumerate(names):
    for threads, blocks in ((64, 256), (256, 256), (256, 512)):
        out = torch.zeros(blocks * threads, dtype=torch.float64, device="cuda")
        cyc = torch.zeros(blocks, dtype=torch.int64, device="cuda")
        lib.probe_snip(v, threads, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(cyc.data_ptr()), blocks, 200)
        print(f"{nm:40s} threads={threads:3d} blocks={blocks:3d} cycles={cyc.float().mean().item():8.0f}")
