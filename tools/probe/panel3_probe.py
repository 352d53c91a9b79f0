"""Panel microbenchmark: shipped panel() vs panel3 variants (tools only)."""
import ctypes, os, numpy as np, torch
here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "libpanel3_probe.so"))
rng = np.random.default_rng(0)
G = rng.standard_normal((16, 16)); A = G @ G.T + 16 * np.eye(16)
L = np.linalg.cholesky(A); Li = np.linalg.inv(L)
Ad = torch.tensor(A.ravel(), dtype=torch.float64, device="cuda")
for v, name in ((0, "product"), (1, "p3 base"), (2, "p3 refine-q"), (3, "p3 row0-first"), (4, "p3 both"), (5, "p5 22122"), (6, "p5 11111"), (7, "p5 00000"), (8, "p5 33222"), (9, "p6 +A, EYE")):
    for blocks in (1, 256, 1024):
        out = torch.zeros(blocks * 272, dtype=torch.float64, device="cuda")
        cyc = torch.zeros(blocks, dtype=torch.int64, device="cuda")
        rc = lib.probe_run(v, ctypes.c_void_p(Ad.data_ptr()), ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(cyc.data_ptr()), blocks, 20)
        o = out[:272].cpu().numpy()
        LiT = np.array([[o[t * 17 + j] for j in range(16)] for t in range(16)])
        err = np.abs(LiT - Li.T).max() / np.abs(Li).max()
        c = cyc.cpu().numpy()
        print(f"{name:28s} blocks={blocks:5d} rc={rc} cycles/panel={np.mean(c % (1 << 40)):8.0f} bad={int((c >> 40).any())} |Linv err|={err:.2e}")
