"""Round-6 diagnostic: the fused kernel's output (u16 passes 1 and 2 of a general map, nothing after)
on a cyclic map at an odd chunk size, repeated, against a two-pass restatement of the reference's
greedy pass (tokenizer.rs:56-93) per chunk.  Prints each mismatch's position, chunk and the
neighbourhood.  Test infrastructure only.

    python tools/diag_r06c.py [--cs 69633] [--reps 20]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def greedy(m, toks):
    out, i, n = [], 0, len(toks)
    while i < n:
        if i + 1 < n and (toks[i], toks[i + 1]) in m:
            out.append(m[(toks[i], toks[i + 1])])
            i += 2
        else:
            out.append(toks[i])
            i += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cs", type=int, default=65536 + 4097)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--seed", type=int, default=44)
    a = ap.parse_args()
    import torch
    import blt_amd
    from blt_amd import _lib, synth
    L = _lib.lib()
    m = {**{(32, c): 32 for c in range(97, 123)}, (300, 301): 302}
    data = synth.text(1 << 20, seed=a.seed)
    cs, n = a.cs, data.size
    exp, starts = [], []
    for c0 in range(0, n, cs):
        starts.append(len(exp))
        exp += greedy(m, greedy(m, data[c0:c0 + cs].tolist()))
    exp = np.array(exp, dtype=np.uint16)
    s = blt_amd.BpeStrategy(m)
    L.blt_debug_set_sparse(0)
    L.blt_debug_set_fused(1)
    L.blt_debug_set_fused_only(1)
    d_in = torch.from_numpy(data).cuda()
    wsb = s.workspace_size(n, cs)
    stream = torch.cuda.current_stream().cuda_stream
    nbad = 0
    for it in range(a.reps):
        d_out = torch.zeros(2 * n, dtype=torch.uint8, device="cuda")
        ws = torch.full((wsb,), 0x5A, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        tok = s.encode_device(d_in.data_ptr(), n, cs, d_out.data_ptr(), ws.data_ptr(), wsb, stream, sync=True)
        torch.cuda.synchronize()
        got = d_out[:2 * tok].cpu().numpy().view(">u2").astype(np.uint16)
        ok = tok == exp.size and np.array_equal(got, exp)
        if not ok:
            nbad += 1
            k = min(got.size, exp.size)
            i = int(np.argmax(got[:k] != exp[:k])) if not np.array_equal(got[:k], exp[:k]) else k
            c = int(np.searchsorted(starts, i, "right")) - 1
            print(f"it{it} fused {L.blt_debug_last_fused()} tok {tok} exp {exp.size} first diff {i} chunk {c} "
                  f"(+{i - starts[c]}) got {got[max(0, i - 3):i + 4].tolist()} exp {exp[max(0, i - 3):i + 4].tolist()}",
                  flush=True)
    print(f"{nbad} of {a.reps} mismatched (cs {cs}, n {n}, chunk token starts {starts[:3]})", flush=True)
    L.blt_debug_set_fused_only(0)


if __name__ == "__main__":
    main()
