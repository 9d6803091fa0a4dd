"""Fused passes 1 + 2 against the two-kernel chain on a general map (f2's `multi` workload by
default): synchronous encode_device (the token count read back), host wall clock, median of reps,
output checked bit-exact against the oracle.  Prints one JSON line per mode.

    python tools/fused_rate.py [--mib 256] [--reps 20] [--map multi|selfval|chain]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--map", default="multi")
    a = ap.parse_args()
    import torch
    import blt_amd
    from blt_amd import _lib, synth
    from oracle import oracle as O
    cs = 16 << 20
    n = a.mib << 20
    if a.map == "chain":   # bench.py's `chain` row: runs of 'a', a 24-level doubling chain
        host = np.full(n, 97, np.uint8)
        m = synth.doubling_chain(24)
    else:
        host = synth.text(n, seed=2)
        m = synth.CHAINED_TEXT_MAP if a.map == "multi" else synth.SELF_VALUED_MAP
    s = blt_amd.BpeStrategy(m)
    d_in = torch.from_numpy(host).cuda()
    d_out = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
    wsb = s.workspace_size(n, cs)
    ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    exp = O.COracle(m).run(host, cs, threads=16)
    for mode in (1, 0, 1, 0):
        _lib.lib().blt_debug_set_fused(mode)
        tok = s.encode_device(d_in.data_ptr(), n, cs, d_out.data_ptr(), ws.data_ptr(), wsb, sp, sync=True)
        used = int(_lib.lib().blt_debug_last_fused())
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            s.encode_device(d_in.data_ptr(), n, cs, d_out.data_ptr(), ws.data_ptr(), wsb, sp, sync=True)
            ts.append(time.perf_counter() - t0)
        ms = 1000 * float(np.median(ts))
        got = d_out[:2 * tok].cpu().numpy()
        algo = n + 2 * tok
        print(json.dumps({"map": a.map, "fused_requested": mode, "fused_used": used, "ms": round(ms, 4),
                          "frac": round(algo / (ms / 1000) / 8e12, 4), "u16_passes": int(_lib.lib().blt_debug_last_u16_passes()),
                          "bit_exact": bool(np.array_equal(got, exp))}), flush=True)
    _lib.lib().blt_debug_set_fused(1)


if __name__ == "__main__":
    main()
