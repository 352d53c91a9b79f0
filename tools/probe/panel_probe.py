"""Panel microbenchmark: cycles per panel() call, one wave per workgroup (tools only)."""
import ctypes, os, numpy as np, torch
here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "libpanel_probe.so"))
A = np.array([[20.0 + r if r == c else 1.0 / (1.0 + abs(r - c)) for c in range(16)] for r in range(16)])
b = 1.0 + np.arange(16)
L = np.linalg.cholesky(A); Li = np.linalg.inv(L); y = Li @ b
for v, name in ((0, "product panel"), (1, "raw v_rsq"), (2, "skeleton (readlane+fma only)"), (3, "dpp row_newbcast"), (4, "dpp skeleton no-nop")):
    for blocks in (256,):
        out = torch.zeros(blocks * 288, dtype=torch.float64, device="cuda")
        cyc = torch.zeros(blocks, dtype=torch.int64, device="cuda")
        rc = lib.probe_panel(v, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(cyc.data_ptr()), blocks, 50)
        o = out[:288].cpu().numpy()
        LiT = np.array([[o[t * 17 + j] for j in range(16)] for t in range(16)])
        err = np.abs(LiT - Li.T).max() if v not in (2, 4) else float("nan")
        erry = np.abs(o[272:288] - y).max() if v not in (2, 4) else float("nan")
        print(f"{name:30s} blocks={blocks:4d} rc={rc} cycles/panel={cyc.float().mean().item():8.0f}  |Linv err|={err:.2e} |y err|={erry:.2e}")
