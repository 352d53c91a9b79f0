"""Hardware probe driver: f64 MFMA layout + rates, via ctypes on torch device memory."""
import ctypes, os, numpy as np, torch
here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "libprobe.so"))
lib.probe_rate.restype = ctypes.c_float
dev = torch.device("cuda:0")
st = torch.cuda.current_stream().cuda_stream
A = np.arange(64, dtype=np.float64).reshape(16, 4) * 0.5 + 1
B = (np.arange(64, dtype=np.float64).reshape(4, 16) ** 1.3)
tA, tB = torch.tensor(A, device=dev), torch.tensor(B, device=dev)
tD = torch.zeros(256, dtype=torch.float64, device=dev)
rc = lib.probe_layout(ctypes.c_void_p(tA.data_ptr()), ctypes.c_void_p(tB.data_ptr()), ctypes.c_void_p(tD.data_ptr()), ctypes.c_void_p(st))
torch.cuda.synchronize()
raw = tD.cpu().numpy().reshape(64, 4)
ref = A @ B
ok = True
for l in range(64):
    for r in range(4):
        row, col = (l >> 4) + 4 * r, l & 15
        if abs(raw[l, r] - ref[row, col]) > 1e-9 * abs(ref[row, col]):
            ok = False
print("layout rc", rc, "guide map (col=l&15,row=(l>>4)+4r) ok:", ok)
if not ok:
    for r in range(4):
        print(r, raw[:20, r])
    print(ref[:4, :8])
out = torch.zeros(256 * 4096, dtype=torch.float64, device=dev)
for which, name in ((0, "mfma_f64_16x16x4"), (1, "v_fma_f64")):
    for blocks in (1024, 4096):
        iters = 2000
        lib.probe_rate(which, ctypes.c_void_p(out.data_ptr()), blocks, 100, ctypes.c_void_p(st))
        ms = lib.probe_rate(which, ctypes.c_void_p(out.data_ptr()), blocks, iters, ctypes.c_void_p(st))
        if which == 0:
            flops = blocks * 4 * iters * 4 * 2 * 16 * 16 * 4  # waves*iters*4mfma*2*M*N*K
        else:
            flops = blocks * 256 * iters * 8 * 2
        print(f"{name} blocks={blocks} ms={ms:.3f} TFLOP/s={flops / ms / 1e9:.2f}")
