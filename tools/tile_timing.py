"""Per-tile phase timing of the byte-pass kernel (s_memtime stamps through the debug hook).

    python tools/tile_timing.py [MiB]
Prints mean/median cycles of phase 1 (lookups + wave functions), phase 2 (tile resolve +
look-back), phase 3 (emission + copy-out) and the look-back window statistics."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import blt_amd  # noqa: E402
from blt_amd import synth  # noqa: E402

TILE = 32768
CHUNK = 16 << 20


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    n = mib << 20
    merges = synth.merges_dict(synth.text_merges_50k(synth.text(64 << 20, seed=3), seed=3))
    s = blt_amd.BpeStrategy(merges)
    d_in = torch.from_numpy(synth.text(n, seed=3)).cuda()
    d_out = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
    wsb = s.workspace_size(n, CHUNK)
    ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    ntiles = (n + TILE - 1) // TILE
    dbg = torch.zeros((8 + 4 * 16) * ntiles, dtype=torch.int64, device="cuda")
    L = blt_amd._lib.lib()
    L.blt_debug_set_tile_record.argtypes = [ctypes.c_void_p]
    sp = torch.cuda.current_stream().cuda_stream
    for it in range(3):
        L.blt_debug_set_tile_record(dbg.data_ptr() if it == 2 else None)
        s.encode_device(d_in.data_ptr(), n, CHUNK, d_out.data_ptr(), ws.data_ptr(), wsb, sp, sync=True)
    L.blt_debug_set_tile_record(None)
    rec = dbg.cpu().numpy().astype(np.int64)
    how = rec[1:4 * ntiles:4] & 0xFFFFFFFF
    st = rec[4 * ntiles:8 * ntiles].reshape(ntiles, 4)
    ok = st[:, 0] != 0
    p1, p2 = st[ok, 1] - st[ok, 0], st[ok, 2] - st[ok, 1]
    for name, v in (("phase1+lookback", p1), ("resolve+emit", p2), ("iteration", p1 + p2)):
        print(f"{name:16s} mean {v.mean():9.0f}  median {np.median(v):9.0f}  p90 {np.percentile(v, 90):9.0f} cycles")
    sp = st[ok, 3]
    print(f"look-back spins mean {sp.mean():.2f} median {np.median(sp)} p90 {np.percentile(sp, 90)} max {sp.max()}")
    wv = rec[8 * ntiles:].reshape(ntiles, -1, 4)
    okw = wv[:, 0, 0] > 0
    wv = wv[okw]
    print("per wave (mean cycles): phase1-work  B1-wait  emit-work  B2-wait")
    for w in range(wv.shape[1]):
        a = wv[:, w, :].mean(axis=0)
        print(f"  wave {w:2d}: {a[0]:8.0f} {a[1]:8.0f} {a[2]:8.0f} {a[3]:8.0f}")
    valid = how != 0xFFFF
    f, qs, rounds = how & 63, (how >> 6) & 3, how >> 8
    print("look-back: first-inclusive lane mean %.1f, window mean %.2f, extra rounds mean %.3f max %d" %
          (f[valid].mean(), qs[valid].mean(), rounds[valid].mean(), rounds[valid].max()))


if __name__ == "__main__":
    main()
