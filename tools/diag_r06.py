"""Round-6 diagnostic: the device API on one general-map case, with the workspace's control block and
chain block printed after the call (torch buffers; the null stream and a torch stream; workspace
prefilled with 0x5A or zeroed).  Test infrastructure: compares with the oracle.

    BLT_LIB_PATH=... python tools/diag_r06.py [--case chained_text] [--cs 4099]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="chained_text")
    ap.add_argument("--cs", type=int, default=4099)
    ap.add_argument("--n", type=int, default=300_001)
    a = ap.parse_args()
    import torch
    import blt_amd
    from blt_amd import _lib, synth
    from oracle import oracle as O
    L = _lib.lib()
    text = synth.text(a.n, seed=5)
    m = synth.CHAINED_TEXT_MAP if a.case == "chained_text" else synth.doubling_chain(8)
    s = blt_amd.BpeStrategy(m)
    cs, n = a.cs, text.size
    exp = O.COracle(m).run(text, cs, threads=8)
    got = s.process_chunks(text, cs)
    print("host path", got.size // 2, "exp", exp.size // 2, "equal", bool(np.array_equal(got, exp)),
          "fused", L.blt_debug_last_fused(), flush=True)
    nch = (n + cs - 1) // cs
    wsb = s.workspace_size(n, cs)
    d_in = torch.from_numpy(text).cuda()
    for stream_kind in ("null", "torch"):
        for fill in (0x5A, 0):
            d_out = torch.zeros(2 * n, dtype=torch.uint8, device="cuda")
            d_off = torch.full((nch + 1,), -1, dtype=torch.int64, device="cuda")
            ws = torch.full((wsb,), fill, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            st = 0 if stream_kind == "null" else torch.cuda.current_stream().cuda_stream
            try:
                tok = s.encode_device(d_in.data_ptr(), n, cs, d_out.data_ptr(), ws.data_ptr(), wsb, st, d_off.data_ptr(),
                                      sync=True)
                err = ""
            except blt_amd.BltError as e:
                tok, err = -1, str(e)[:200]
                s.clear_error()
            torch.cuda.synchronize()
            ctl = ws[:64].cpu().numpy().view(np.uint32)
            ntiles = (n + 32767) // 32768
            zb = (64 + 8 * ntiles + 15) // 16 * 16
            chain = ws[zb:zb + 48].cpu().numpy()
            ok = tok * 2 == exp.size and bool(np.array_equal(d_out[:exp.size].cpu().numpy(), exp))
            print(stream_kind, hex(fill), "tok", tok, "ok", ok, "fused", L.blt_debug_last_fused(), err, flush=True)
            print("  ctl", ctl[:10].tolist())
            print("  chain u64", chain[:32].view(np.uint64).tolist(), "fin_gate", int(chain[32:36].view(np.uint32)[0]))


if __name__ == "__main__":
    main()
