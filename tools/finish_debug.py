"""Reproduces test_gpu_fused.py::test_fused_halo_fallback's first map on the two-kernel chain with
the finish kernels, and prints the finish kernel's per-group records (tests only: the debug hook)
against the oracle's per-chunk counts, and the group status words.

    python tools/finish_debug.py
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import blt_amd
    from oracle import oracle as O
    L = blt_amd._lib.lib()
    L.blt_debug_set_fused(0)
    cs = 4096 * 3 + 7
    data = np.frombuffer(b"ab" * ((1 << 19) + 3), np.uint8).copy()
    data[::5003] = 99
    m = {(97, 98): 256, (98, 97): 257, (256, 256): 258, (258, 99): 259}
    s = blt_amd.BpeStrategy(m)
    n = data.size
    nch = (n + cs - 1) // cs
    exp, elens = O.COracle(m).run(data, cs, threads=8, return_lens=True)
    d_in = torch.from_numpy(data).cuda()
    d_out = torch.zeros(2 * n, dtype=torch.uint8, device="cuda")
    d_off = torch.zeros(nch + 1, dtype=torch.int64, device="cuda")
    wsb = s.workspace_size(n, cs)
    ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    dbg = torch.zeros(16 * nch + 64, dtype=torch.int64, device="cuda")
    L.blt_debug_set_tile_record.argtypes = [ctypes.c_void_p]
    L.blt_debug_set_tile_record(dbg.data_ptr())
    st = torch.cuda.current_stream().cuda_stream
    for rep in range(3):
        dbg.zero_()
        try:
            tok = s.encode_device(d_in.data_ptr(), n, cs, d_out.data_ptr(), ws.data_ptr(), wsb, st, d_chunk_off=d_off.data_ptr())
            ok = 2 * tok == exp.size and np.array_equal(d_out[:2 * tok].cpu().numpy(), exp)
            print("rep", rep, "tokens", tok, "ok", ok)
        except blt_amd.BltError as e:
            print("rep", rep, "error", e)
            s.clear_error()
        torch.cuda.synchronize()
        rec = dbg.cpu().numpy().reshape(-1, 16)
        final = np.cumsum(np.concatenate([[0], elens // 2]))
        def fmt(w):
            w = int(w) & ((1 << 64) - 1)
            return f"{w >> 62}:{(w >> 60) & 3}:{w & ((1 << 30) - 1)}:{(w >> 30) & ((1 << 29) - 1)}:{w & ((1 << 60) - 1)}"
        for r in rec[:12]:
            if r[6] == 0:
                continue
            g, S, n0, nf, Og, cw, lg, nc = (int(x) for x in r[:8])
            print("   status g-1", fmt(r[8]), "g0", fmt(r[9]), "g", fmt(r[10]), "g-2", fmt(r[11]))
            grp = lg >> 32
            c0, c1 = g * grp, min(g * grp + grp, nch)
            print(f"g {g:3d} S {S:8d} n0 {n0:6d} n {nf:6d} O {Og:12d} expO {int(final[c0]):8d} expn {int(final[c1] - final[c0]):6d} "
                  f"C {cw & 255} how {(cw >> 8) & 0xFFFFFF:#x} spins {cw >> 32} lmax {lg & 0xFFFFFFFF} grp {grp} nc {nc}")
    L.blt_debug_set_tile_record(None)


if __name__ == "__main__":
    main()
