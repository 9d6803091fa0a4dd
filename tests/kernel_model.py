"""Lane-exact CPU model of merge_pass_kernel (blt_amd/csrc/bpe_kernels.hip), for tests only.

It reproduces the kernel's decomposition — 16-position lane segments, wave ballots and
prefix scans, per-(sub-tile, wave) group functions, the tile function, and the look-back
composition (done serially here) — so the algebra of the parallel scan can be checked against
the sequential oracle on CPU, without a GPU.
"""
from typing import Dict, Tuple

THREADS, SEG, SUB = 512, 16, 4
WAVES = THREADS // 64
SUBPOS = THREADS * SEG
TILEPOS = SUB * SUBPOS


def merges_for(m, c):
    mc = m if c else (m & ~1)
    s = mc & ~(mc << 1)
    rodd = mc & ~(mc + (s & 0xAAAA))
    return (mc & ~rodd & 0x5555) | (rodd & 0xAAAA)


def lands_for(M, c, valid):
    return ~((M << 1) | (c ^ 1)) & valid & 0xFFFF


def resolve(items):
    """items: per-lane (ident, cout, cnt0, cnt1) for 64 lanes -> per-lane (has_below, below_cout,
    excl0, excl1) and the wave function (ident, cout, cnt0, cnt1)."""
    out = []
    last_nonid_cout = None
    acc0 = acc1 = 0
    for ident, cout, c0, c1 in items:
        hb = last_nonid_cout is not None
        bc = last_nonid_cout if hb else 0
        cin0 = bc if hb else 0
        cin1 = bc if hb else 1
        out.append((hb, bc, acc0, acc1))
        acc0 += c1 if cin0 else c0
        acc1 += c1 if cin1 else c0
        if not ident:
            last_nonid_cout = cout
    fn = (last_nonid_cout is None, last_nonid_cout or 0, acc0, acc1)
    return out, fn


def run_pass(seq, merges: Dict[Tuple[int, int], int], chunk_size: int):
    """One kernel pass over positions `seq` (ints) -> output tokens."""
    n = len(seq)
    out = [None] * n
    C, O = 1, 0
    ntiles = (n + TILEPOS - 1) // TILEPOS
    for T in range(ntiles):
        tile0 = T * TILEPOS
        lanes = {}
        wfn = {}
        for j in range(SUB):
            sub0 = tile0 + j * SUBPOS
            for w in range(WAVES):
                items = []
                for l in range(64):
                    pos = sub0 + (w * 64 + l) * SEG
                    vmask = 0 if pos >= n else (0xFFFF if n - pos >= 16 else (1 << (n - pos)) - 1)
                    m = 0
                    vals = [0] * 16
                    for k in range(16):
                        p = pos + k
                        if p + 1 < n:
                            v = merges.get((seq[p], seq[p + 1]))
                            if v is not None:
                                m |= 1 << k
                                vals[k] = v
                    # the kernel's boundary walk: chunk starts b in (sub0, sub0 + SUBPOS] clear m at b - 1
                    x = sub0 + 1 if sub0 + 1 < n else n
                    kk = (x + chunk_size - 1) // chunk_size
                    b = min(kk * chunk_size, n)
                    while b < n and b <= sub0 + SUBPOS:
                        e = b - 1
                        if pos <= e < pos + 16:
                            m &= ~(1 << (e - pos))
                        b = min((kk + 1) * chunk_size, n)
                        kk += 1
                    ident = m == 0xFFFF
                    M1, M0 = merges_for(m, 1), merges_for(m, 0)
                    cnt1 = bin(lands_for(M1, 1, vmask)).count("1")
                    cnt0 = bin(lands_for(M0, 0, vmask)).count("1")
                    cout = ((M1 >> 15) & 1) ^ 1
                    items.append((ident, cout, cnt0, cnt1))
                    lanes[(j, w, l)] = (pos, m, vmask, vals)
                res, fn = resolve(items)
                for l in range(64):
                    lanes[(j, w, l)] = lanes[(j, w, l)] + res[l]
                wfn[(j, w)] = fn
        groups = [wfn[(j, w)] for j in range(SUB) for w in range(WAVES)]
        gres, tf = resolve(groups + [(True, 0, 0, 0)] * (64 - len(groups)))
        # look-back (serial): the carry/offset entering this tile are C, O
        tile_cnt = tf[3] if C else tf[2]
        for j in range(SUB):
            for w in range(WAVES):
                g = j * WAVES + w
                ghb, gbc, gx0, gx1 = gres[g]
                cg = gbc if ghb else C
                og = gx1 if C else gx0
                for l in range(64):
                    pos, m, vmask, vals, hb, bc, e0, e1 = lanes[(j, w, l)]
                    c = bc if hb else cg
                    lane_off = og + (e1 if cg else e0)
                    M = merges_for(m, c)
                    L = lands_for(M, c, vmask)
                    r = O + lane_off
                    for k in range(16):
                        if (L >> k) & 1:
                            out[r] = vals[k] if (M >> k) & 1 else seq[pos + k]
                            r += 1
        co = (1 if C else 0) if tf[0] else tf[1]
        O += tile_cnt
        C = co
    return out[:O]
