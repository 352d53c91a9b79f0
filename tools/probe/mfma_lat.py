import ctypes, os, torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmfma_lat.so"))
out = torch.zeros(64, dtype=torch.float64, device="cuda"); cyc = torch.zeros(1, dtype=torch.int64, device="cuda")
for which in (1, 2, 4, 8, 0):
    iters = 1000
    lib.run(which, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(cyc.data_ptr()), iters)
    lib.run(which, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(cyc.data_ptr()), iters)
    c = cyc.item()
    if which:
        print(f"{which} interleaved chain(s): {c / (iters * 4 * which):.1f} cycles per MFMA, {c / (iters * 4):.1f} per chain step")
    else:
        print(f"LDS dependent read: {c / iters:.1f} cycles per load->use")
