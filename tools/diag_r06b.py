"""Round-6 diagnostic: a cyclic general map at an odd chunk size, encoded repeatedly through the
device API (sync and async, 0x5A workspace) under each blt_debug_set_u16_chain mode (bit 0: chained
chunk maps, bit 1: the host's extended scan bound).  Prints per mode the mismatching runs, the first
mismatching token and the pass counts.  Test infrastructure: compares with the oracle.

    python tools/diag_r06b.py [--cs 69633] [--reps 6] [--modes 3,1,2,0]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cs", type=int, default=65536 + 4097)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--modes", default="3,1,2,0")
    ap.add_argument("--mib", type=int, default=1)
    ap.add_argument("--fused", default="1,0", help="blt_debug_set_fused values to run")
    a = ap.parse_args()
    import torch
    import blt_amd
    from blt_amd import _lib, synth
    from oracle import oracle as O
    L = _lib.lib()
    m = {**{(32, c): 32 for c in range(97, 123)}, (300, 301): 302}
    data = synth.text(a.mib << 20, seed=44)
    cs, n = a.cs, data.size
    exp, elens = O.COracle(m).run(data, cs, threads=16, return_lens=True)
    eoff = np.concatenate([[0], np.cumsum(elens // 2)])
    s = blt_amd.BpeStrategy(m)
    L.blt_debug_set_sparse(0)
    d_in = torch.from_numpy(data).cuda()
    wsb = s.workspace_size(n, cs)
    nch = (n + cs - 1) // cs
    stream = torch.cuda.current_stream().cuda_stream
    has_modes = hasattr(L, "blt_debug_set_u16_chain")
    combos = [(f, md) for f in [int(x) for x in a.fused.split(",")]
              for md in ([int(x) for x in a.modes.split(",")] if has_modes else [-1])]
    print("chunk token offsets (oracle):", eoff[:4].tolist(), "...", flush=True)
    for fused, mode in combos:
        L.blt_debug_set_fused(fused)
        if has_modes:
            L.blt_debug_set_u16_chain(mode)
        bad = []
        for it in range(a.reps):
            for sync in (True, False):
                d_out = torch.zeros(2 * n, dtype=torch.uint8, device="cuda")
                d_off = torch.full((nch + 1,), -1, dtype=torch.int64, device="cuda")
                ws = torch.full((wsb,), 0x5A, dtype=torch.uint8, device="cuda")
                torch.cuda.synchronize()
                s.encode_device(d_in.data_ptr(), n, cs, d_out.data_ptr(), ws.data_ptr(), wsb, stream, d_off.data_ptr(),
                                sync=sync)
                torch.cuda.synchronize()
                got = d_out[:exp.size].cpu().numpy()
                passes = int(L.blt_debug_last_u16_passes())
                scans = int(L.blt_debug_last_scan_passes()) if hasattr(L, "blt_debug_last_scan_passes") else -1
                lf = int(L.blt_debug_last_fused())
                if not np.array_equal(got, exp):
                    g16, e16 = got.view(">u2"), exp.view(">u2")
                    i = int(np.argmax(g16 != e16))
                    off = d_off.cpu().numpy()
                    bad.append(f"it{it} sync={sync} first token {i} (chunk {int(np.searchsorted(eoff, i, 'right')) - 1}) "
                               f"got {g16[max(0, i - 2):i + 3].tolist()} exp {e16[max(0, i - 2):i + 3].tolist()} "
                               f"offsets {off[:4].tolist()} passes {passes} scans {scans} fused {lf}")
        print(f"fused {fused} mode {mode}: {len(bad)} of {2 * a.reps} mismatched; last passes {passes} scans {scans} "
              f"fused ran {lf}", flush=True)
        for b in bad[:6]:
            print("   ", b, flush=True)
    if has_modes:
        L.blt_debug_set_u16_chain(3)
    L.blt_debug_set_fused(1)


if __name__ == "__main__":
    main()
