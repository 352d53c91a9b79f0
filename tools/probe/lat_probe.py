"""Dependent-latency microbenchmarks (tools only): cycles per op in a 64-op chain."""
import ctypes, os, torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblat_probe.so"))
out = torch.zeros(1024, dtype=torch.float64, device="cuda"); cyc = torch.zeros(16, dtype=torch.int64, device="cuda")
names = ["v_fma_f64", "v_rsq_f64 + add", "2 v_readlane + mul", "MFMA f64 16x16x4 (acc chain)", "MFMA -> A operand",
         "2 v_permlane16_swap + mul", "v_mul_f64", "v_rcp_f64 + add", "MFMA -> VALU mul -> MFMA",
         "tput v_fma_f64 (8 chains)", "tput v_fmac_f64_dpp newbcast", "tput v_fmac_f64 (asm)", "tput fmac_dpp row_mask 1", "tput v_mul_f64",
         "tput v_mov_b32", "tput v_mov_b64", "tput v_permlane16_swap", "tput v_readlane_b32", "tput v_cmp_class_f64",
         "tput v_add_u32", "tput s_add_u32", "tput v_rsq_f64", "tput v_mov_b32_dpp", "s_nop 0", "s_nop 1", "v_mov_b32 + s_nop 1"]
print("waves per SIMD:                      1        2        4")
for w, nm in enumerate(names):
    row = []
    for nt in (64, 512, 1024):
        for _ in range(3):
            lib.lat_run(w, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(cyc.data_ptr()), nt)
        row.append(cyc[: nt // 64].double().mean().item() / 64)
    print(f"{nm:32s} " + " ".join(f"{v:8.1f}" for v in row) + "  cycles/op per wave")
# dependent global loads: lane l follows its own chain, stride 33 ints (distinct lines)
for n in (2048, 1 << 16, 1 << 20, 1 << 26):
    idx = (torch.arange(n, dtype=torch.int64) + 64 * 33) % n
    buf = idx.to(torch.int32).cuda()
    o = torch.zeros(64, dtype=torch.int32, device="cuda")
    for _ in range(2):
        lib.chase_run(ctypes.c_void_p(buf.data_ptr()), 256, ctypes.c_void_p(o.data_ptr()), ctypes.c_void_p(cyc.data_ptr()))
    print(f"pointer chase over {n * 4 / 1024:9.0f} KB: {cyc[0].item():6d} cycles per dependent load")
