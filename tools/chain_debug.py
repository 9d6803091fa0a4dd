"""Debug aid for chain launches (round 4): one general-map case run through the device API with
chain launches and finish kernels on and off, each combination reporting the error message (with
the control block's flags) or whether the tokens and chunk offsets match the oracle.

    python tools/chain_debug.py [--case doubling] [--mib 4]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="doubling")
    ap.add_argument("--mib", type=int, default=4)
    ap.add_argument("--cs", type=int, default=1 << 20)
    ap.add_argument("--depth", type=int, default=16)
    a = ap.parse_args()
    import torch
    import blt_amd
    from blt_amd import synth
    from oracle import oracle as O
    L = blt_amd._lib.lib()
    rng = np.random.default_rng(7)
    if a.case == "doubling":
        m = synth.doubling_chain(a.depth)
        data = np.full((a.mib << 20) + 77, 97, np.uint8)
        data[rng.choice(data.size, 40, replace=False)] = 98
    else:
        m = synth.SELF_VALUED_MAP
        data = synth.text((a.mib << 20) + 5, seed=17)
    cs = a.cs
    exp, elens = O.COracle(m).run(data, cs, threads=8, return_lens=True)
    n = data.size
    nch = (n + cs - 1) // cs
    print(f"case {a.case}: n {n}, cs {cs}, {nch} chunks, expected tokens {exp.size // 2}")
    d_in = torch.from_numpy(data).cuda()
    stream = torch.cuda.current_stream().cuda_stream
    for chain_on in (1, 0):
        for fin_on in (1, 0):
            L.blt_debug_set_chain(chain_on)
            L.blt_debug_set_finish(fin_on)
            s = blt_amd.BpeStrategy(m)
            d_out = torch.zeros(2 * n, dtype=torch.uint8, device="cuda")
            d_off = torch.full((nch + 1,), -1, dtype=torch.int64, device="cuda")
            wsb = s.workspace_size(n, cs)
            ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
            tag = f"chain={chain_on} finish={fin_on}"
            try:
                tok = s.encode_device(d_in.data_ptr(), n, cs, d_out.data_ptr(), ws.data_ptr(), wsb, stream,
                                      d_off.data_ptr(), sync=True)
                torch.cuda.synchronize()
                got = d_out[:2 * tok].cpu().numpy()
                offs = d_off.cpu().numpy()
                ok = got.size == exp.size and np.array_equal(got, exp)
                okl = np.array_equal(np.diff(offs) * 2, elens)
                first_bad = -1
                if not ok:
                    k = min(got.size, exp.size)
                    diff = np.nonzero(got[:k] != exp[:k])[0]
                    first_bad = int(diff[0]) if diff.size else k
                print(f"{tag}: tokens {tok} (exp {exp.size // 2}) bit-exact {ok} offsets {okl} first diff byte {first_bad} "
                      f"passes {L.blt_debug_last_u16_passes()}")
                if not okl:
                    print("   got offs", offs[:8].tolist(), "exp", np.concatenate([[0], np.cumsum(elens // 2)])[:8].tolist())
            except Exception as e:   # noqa: BLE001
                print(f"{tag}: ERROR {e}")
            s.close()
    L.blt_debug_set_chain(1)
    L.blt_debug_set_finish(1)


if __name__ == "__main__":
    main()
