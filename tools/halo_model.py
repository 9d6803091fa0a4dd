"""Model of halo-resolved carries for a fused pass-1 + pass-2 kernel (design study).

A greedy pass restarts at every pair it does not merge: L[i + 1] = 1 whenever m[i] = 0 (and at
every chunk start).  So the carry into a wave range (is its first byte consumed by a pass-1 merge;
is its first pass-1 token consumed by a pass-2 merge) follows from a short halo of the bytes
before it, as soon as the halo holds a pass-1 restart and, after it, a pass-2 restart.  This
model computes both carries from an H-byte halo for every 1024-byte wave range, checks them
against whole-buffer greedy passes (tokenizer.rs:63-81 restated, per chunk), and reports how often
the halo holds no restart (the cases a kernel would hand to the present two-kernel path).

    python tools/halo_model.py [--mib 2] [--halo 16,32,64] [--maps multi,selfval,cfg2]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

RANGE = 1024


def greedy(seq, starts, lookup):
    """One greedy pass over seq with chunk starts (a set of indices): landing flags, merge flags
    (per index, meaningful where it lands) and the emitted tokens with the index each starts at."""
    n = len(seq)
    land = np.zeros(n, bool)
    merged = np.zeros(n, bool)
    toks, pos = [], []
    i = 0
    while i < n:
        land[i] = True
        v = None
        if i + 1 < n and (i + 1) not in starts:
            v = lookup.get((int(seq[i]), int(seq[i + 1])))
        if v is not None:
            merged[i] = True
            toks.append(v)
            pos.append(i)
            i += 2
        else:
            toks.append(int(seq[i]))
            pos.append(i)
            i += 1
    return land, merged, np.array(toks, np.int64), np.array(pos, np.int64)


def halo_carries(b, ws, H, cs, lookup):
    """(C1, C2, first pass-1 token at or after ws) from bytes [ws - H, ws + 3) only, or None
    when the halo holds no pass-1 restart or, after it, no pass-2 restart."""
    h0 = max(0, ws - H)
    hi = min(len(b), ws + 3)

    def cstart(i):
        return i % cs == 0

    def m1(i):   # pair (i, i + 1) merges in pass 1
        return i + 1 < hi and not cstart(i + 1) and (int(b[i]), int(b[i + 1])) in lookup

    r0 = None
    for i in range(h0, ws + 1):
        if i == 0 or cstart(i) or (i - 1 >= h0 and not m1(i - 1)):
            r0 = i
            break
    if r0 is None:
        return None
    # pass 1 from the restart: landings and tokens up to the first landing at or after ws
    toks, pos = [], []
    i = r0
    while True:
        mg = m1(i)
        toks.append(lookup[(int(b[i]), int(b[i + 1]))] if mg else int(b[i]))
        pos.append(i)
        if i >= ws:
            break
        i += 2 if mg else 1
    c1 = 1 if pos[-1] > ws else 0
    # pass 2 over those tokens: the first restart, then greedy to the last token (the range's first)
    k = len(toks) - 1

    def m2(j):
        return j + 1 <= k and not cstart(pos[j + 1]) and (toks[j], toks[j + 1]) in lookup

    s0 = None
    for j in range(0, k + 1):
        if cstart(pos[j]) or pos[j] == 0 or (j >= 1 and not m2(j - 1)):
            s0 = j
            break
    if s0 is None:
        return None
    j = s0
    while j < k:
        j += 2 if m2(j) else 1
    c2 = 1 if j > k else 0
    return c1, c2, toks[k]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=float, default=2)
    ap.add_argument("--halo", default="16,32,64")
    ap.add_argument("--maps", default="multi,selfval,cfg2")
    ap.add_argument("--cs", type=int, default=1 << 20)
    a = ap.parse_args()
    from blt_amd import synth
    n = int(a.mib * (1 << 20))
    b = synth.text(n, seed=2)
    maps = {"multi": synth.CHAINED_TEXT_MAP, "selfval": synth.SELF_VALUED_MAP,
            "cfg2": synth.merges_dict(synth.top_pair_merges(b, 256))}
    cs = a.cs
    starts = set(range(0, n, cs))
    for name in a.maps.split(","):
        lookup = maps[name]
        land1, _, t1, p1 = greedy(b, starts, lookup)
        tstarts = set(np.nonzero(np.isin(p1, list(starts)))[0].tolist())
        land2, _, _, _ = greedy(t1, tstarts, lookup)
        first_tok = np.searchsorted(p1, np.arange(0, n, RANGE))
        for H in [int(x) for x in a.halo.split(",")]:
            fail = bad = 0
            for r, ws in enumerate(range(RANGE, n, RANGE)):
                res = halo_carries(b, ws, H, cs, lookup)
                if res is None:
                    fail += 1
                    continue
                c1, c2, tok = res
                j = first_tok[r + 1]
                if c1 != (0 if land1[ws] else 1) or tok != t1[j] or c2 != (0 if land2[j] else 1):
                    bad += 1
            total = n // RANGE - 1
            print(f"{name:8s} halo {H:3d} B: {total} wave ranges, {fail} without restarts "
                  f"({100.0 * fail / total:.3f} %), {bad} wrong")


if __name__ == "__main__":
    main()
