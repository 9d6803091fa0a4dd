"""Per-tile phase timing of the byte-pass kernel (s_memtime stamps through the debug hook, in
the timing build build/xp/libblt_bpe_timing.so from `make exp`, or BLT_LIB_PATH).

    python tools/tile_timing.py [MiB] [--random] [--few]   (--random: cfg5's random bytes instead of cfg3's
    text; --few: a two-merge map, ~1 token per byte)
Prints mean/median cycles of phase 1 (lookups + wave functions), phase 2 (tile resolve +
look-back), phase 3 (emission + copy-out) and the look-back window statistics."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the stamps exist only in the timing build of the kernel (make exp; -DBLT_TIMING)
os.environ.setdefault("BLT_LIB_PATH", os.path.join(ROOT, "build", "xp", "libblt_bpe_timing.so"))
import torch  # noqa: E402

import blt_amd  # noqa: E402
from blt_amd import synth  # noqa: E402

TILE = 32768
CHUNK = 16 << 20


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    mib = int(args[0]) if args else 1024
    n = mib << 20
    if "--few" in sys.argv:   # two merges ("e ", "th"): ~0.97 tokens per byte, two-part emission
        merges = {(101, 32): 256, (116, 104): 257}
    elif "--cfg2" in sys.argv:   # cfg2's 256 merges ranked from its text (seed 2)
        merges = synth.merges_dict(synth.top_pair_merges(synth.text(100 << 20, seed=2), 256))
    else:
        merges = synth.merges_dict(synth.text_merges_50k(synth.text(64 << 20, seed=3), seed=3))
    s = blt_amd.BpeStrategy(merges)
    data = synth.random_bytes(n, seed=5) if "--random" in sys.argv else \
        synth.text(n, seed=2 if "--cfg2" in sys.argv else 3)   # cfg5 / cfg2 / cfg3
    d_in = torch.from_numpy(data).cuda()
    d_out = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
    wsb = s.workspace_size(n, CHUNK)
    ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    ntiles = (n + TILE - 1) // TILE
    dbg = torch.zeros((8 + 8 * 16) * ntiles + 4 * 4096, dtype=torch.int64, device="cuda")
    L = blt_amd._lib.lib()
    L.blt_debug_set_tile_record.argtypes = [ctypes.c_void_p]
    sp = torch.cuda.current_stream().cuda_stream
    for it in range(3):
        L.blt_debug_set_tile_record(dbg.data_ptr() if it == 2 else None)
        s.encode_device(d_in.data_ptr(), n, CHUNK, d_out.data_ptr(), ws.data_ptr(), wsb, sp, sync=True)
    L.blt_debug_set_tile_record(None)
    rec = dbg.cpu().numpy().astype(np.int64)
    # workgroup start / table copied / exit (s_memrealtime, 100 MHz) against the tiles' publishes
    wg = rec[(8 + 8 * 16) * ntiles:].reshape(-1, 4)
    wg = wg[wg[:, 0] > 0]
    if wg.size:
        t0 = wg[:, 0].min()
        us_ = lambda v: (v - t0) / 100.0
        pubs = rec[4 * ntiles:8 * ntiles:4]
        pubs = pubs[pubs > 0]
        print(f"{len(wg)} workgroups: start us p50 {np.median(us_(wg[:, 0])):.2f} max {us_(wg[:, 0]).max():.2f}; "
              f"table copied p50 {np.median(us_(wg[:, 1])):.2f} max {us_(wg[:, 1]).max():.2f}; "
              f"exit p50 {np.median(us_(wg[:, 2])):.2f} max {us_(wg[:, 2]).max():.2f}; "
              f"tile publishes first {us_(pubs.min()):.2f} last {us_(pubs.max()):.2f}")
        ex = np.sort(us_(wg[:, 2]))
        print("  exit us percentiles p0 %.2f p10 %.2f p50 %.2f p90 %.2f p100 %.2f; start p0 %.2f p100 %.2f" %
              (ex[0], np.percentile(ex, 10), np.median(ex), np.percentile(ex, 90), ex[-1],
               us_(wg[:, 0]).min(), us_(wg[:, 0]).max()))
        ps = np.sort(us_(pubs))
        print("  tile publishes: first 256 done by %.2f us, last 256 start at %.2f us; mean gap per 256 tiles %.3f us" %
              (ps[min(255, ps.size - 1)], ps[max(0, ps.size - 256)], (ps[-1] - ps[0]) / max(1, ps.size / 256)))
    how = rec[1:4 * ntiles:4] & 0xFFFFFFFF
    wv8 = rec[8 * ntiles:(8 + 8 * 16) * ntiles].reshape(ntiles, 16, 8)
    wv = wv8[:, :, :6]
    ok = wv[:, 0, :].sum(axis=1) > 0
    wv = wv[ok]
    sub = wv8[ok][:, :, 6:8]
    names = ["x-wait", "phase1", "lb+pub", "lb-wait", "emit", "tk-wait"]
    print("per wave mean cycles: " + " ".join(f"{x:>8s}" for x in names) + "     total")
    for w in range(16):
        m = wv[:, w, :].mean(axis=0)
        print(f"  wave {w:2d}:          " + " ".join(f"{v:8.0f}" for v in m) + f"  {m.sum():8.0f}")
    print("phase 1 split (lookups+masks | lane functions, lgkmcnt drained): " +
          " ".join(f"w{w}:{sub[:, w, 0].mean():.0f}|{sub[:, w, 1].mean():.0f}" for w in range(16)))
    sp = rec[4 * ntiles + 3:8 * ntiles:4] & 0xFFFFFFFF
    bad = rec[4 * ntiles + 3:8 * ntiles:4] >> 32
    print(f"look-back spins mean {sp.mean():.2f} max {sp.max()}")
    # s_memrealtime (100 MHz, one clock for the whole chip): aggregate publish of each tile,
    # look-back snapshot issue and completion of its successor's look-back
    pub = rec[4 * ntiles:8 * ntiles:4]
    snap = rec[4 * ntiles + 1:8 * ntiles:4] & 0xFFFFFFFF
    done = (rec[4 * ntiles + 1:8 * ntiles:4] >> 32) & 0xFFFFFFFF
    pub32 = pub & 0xFFFFFFFF
    t = np.arange(2, ntiles)
    gap = ((snap[t] - pub32[t - 1] + (1 << 31)) % (1 << 32)) - (1 << 31)   # snapshot - predecessor publish
    wait = ((done[t] - snap[t] + (1 << 31)) % (1 << 32)) - (1 << 31)
    spt = sp[t]
    us = lambda v: v / 100.0
    for k in range(0, 4):
        sel = spt == k if k < 3 else spt >= 3
        if sel.any():
            print(f"spins {k}{'+' if k == 3 else ' '}: {sel.sum():6d} tiles; snapshot - pred publish us "
                  f"p10 {us(np.percentile(gap[sel], 10)):6.2f} p50 {us(np.median(gap[sel])):6.2f} "
                  f"p90 {us(np.percentile(gap[sel], 90)):6.2f}; look-back us p50 {us(np.median(wait[sel])):6.2f}")
    hist = np.histogram(us(gap), bins=[-100, -4, -2, -1, 0, 1, 2, 3, 4, 6, 8, 100])
    print("gap histogram (us):", list(zip(hist[1][:-1].tolist(), hist[0].tolist())))
    # spin probability as a function of the gap
    for lo, hi in [(-100, 0), (0, 1), (1, 2), (2, 3), (3, 4), (4, 6), (6, 100)]:
        sel = (us(gap) >= lo) & (us(gap) < hi)
        if sel.any():
            print(f"  gap [{lo},{hi}) us: n {sel.sum():6d}, P(spin) {(spt[sel] > 0).mean():.2f}")
    # the first tile found not ready: its distance back, and its publish time vs the snapshot
    sel = np.nonzero(bad[t] > 0)[0]
    if sel.size:
        tt = t[sel]
        d = bad[tt]
        print("first not-ready tile distance: p10 %d p50 %d p90 %d max %d; share at distance 1: %.2f" %
              (np.percentile(d, 10), np.median(d), np.percentile(d, 90), d.max(), (d == 1).mean()))
        src = tt - d
        okk = src >= 0
        g2 = ((snap[tt[okk]] - pub32[src[okk]] + (1 << 31)) % (1 << 32)) - (1 << 31)
        print("  its publish vs snapshot (snapshot - publish) us: p10 %.2f p50 %.2f p90 %.2f" %
              (us(np.percentile(g2, 10)), us(np.median(g2)), us(np.percentile(g2, 90))))
    valid = how != 0xFFFF
    f, qs, rounds = how & 63, (how >> 6) & 3, how >> 8
    print("look-back: first-inclusive lane mean %.1f, window mean %.2f, extra rounds mean %.3f max %d" %
          (f[valid].mean(), qs[valid].mean(), rounds[valid].mean(), rounds[valid].max()))


if __name__ == "__main__":
    main()
