"""Sequential restatement of the sparse passes (bpe_kernels.hip, sparse_region_kernel and
sparse_apply_kernel: seeds, run owners, greedy walks, hole bitmap) checked against the oracle:
a few full passes, then sparse passes until no live token is made (at most 250), then full passes
from the compacted state; asserts that no merge is made twice and that the applied merges equal
the holes (the compaction's counts).  Debug aid, small inputs only.

    CASE=long_tail|rndSEED FULL=<full passes first> CS=<chunk bytes> python tools/sparse_sim.py
"""
import os
import sys
import zlib

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
case = os.environ.get("CASE", "long_tail")
rng = np.random.default_rng(zlib.crc32(case.encode()))
if case == "long_tail":
    m = {(97, 98): 97, (99, 99): 256}
    parts, size = [], 0
    while size < (1 << 16):
        k = int(rng.integers(1, 300)) if rng.random() < 0.02 else int(rng.integers(0, 8))
        parts.append(np.frombuffer(b"a" + b"b" * k + b"cc" * int(rng.integers(0, 3)), np.uint8)); size += parts[-1].size
    parts.append(np.frombuffer(b"a" + b"b" * 270, np.uint8))
    data = np.concatenate(parts)
else:
    seed = int(case[3:])
    rng = np.random.default_rng(seed)
    m = {}
    for i, (a, b) in enumerate(rng.integers(97, 101, (10, 2))):
        m.setdefault((int(a), int(b)), int(rng.integers(97, 101)) if i % 2 else 256 + i)
    for i in range(12):
        a, b = int(rng.integers(256, 266)), int(rng.integers(97, 101))
        m.setdefault((a, b), int(rng.integers(97, 101)))
    data = rng.integers(97, 101, 1 << 14, dtype=np.uint8)
cs = int(os.environ.get('CS', 1 << 14))
exp = O.COracle(m).run(data, cs, threads=1)
expt = exp.view('>u2').astype(np.int64)
# full greedy pass over token list per chunk
comp = set()
for (a, b), v in m.items(): comp.add(a); comp.add(b)
def greedy(toks):
    out = []; i = 0; merged = 0; live = False
    while i < len(toks):
        if i + 1 < len(toks) and (toks[i], toks[i+1]) in m:
            v = m[(toks[i], toks[i+1])]; out.append(v); i += 2; merged += 1; live |= v in comp
        else:
            out.append(toks[i]); i += 1
    return out, merged
chunks = [list(data[i:i+cs]) for i in range(0, len(data), cs)]
# pass 1 .. 6 full
for p in range(int(os.environ.get('FULL', '6'))):
    chunks = [greedy(c)[0] for c in chunks]
# sparse from here
tok = [t for c in chunks for t in c]
N = len(tok)
cst = set(); o = 0
for c in chunks: cst.add(o); o += len(c)
holes = [False] * N
def nxt(p):
    p += 1
    while p < N and holes[p]: p += 1
    return p
def prv(p):
    p -= 1
    while p >= 0 and holes[p]: p -= 1
    return p
seeds = [p for p in range(N - 1) if (p + 1) not in cst and (tok[p], tok[p+1]) in m]
H = 0
for ps in range(250):
    if not seeds: break
    bits = set(seeds); merges = []; out = []
    for sd in seeds:
        a = sd; owner = True
        while True:
            if a in cst: break
            pq = prv(a)
            if pq < 0 or (tok[pq], tok[a]) not in m: break
            if pq in bits: owner = False; break
            a = pq
        if not owner: continue
        i = a
        while True:
            j = nxt(i)
            if j >= N or j in cst: break
            if (tok[i], tok[j]) not in m: break
            v = m[(tok[i], tok[j])]
            merges.append((i, j, v))
            if v in comp: out.append(i)
            k = nxt(j)
            if k >= N or k in cst: break
            if (tok[j], tok[k]) not in m: break
            i = k
    js = [j for _, j, _ in merges]
    assert len(js) == len(set(js)), ("dup j", ps)
    for i, j, v in merges:
        assert not holes[j]
        tok[i] = v; holes[j] = True; H += 1
    assert len(out) == len(set(out)), ("dup seeds", ps, len(out), len(set(out)))
    seeds = out
print("passes", ps, "H", H, "holes", sum(holes))
# finish with full passes from the compacted state, then compare
res = [tok[p] for p in range(N) if not holes[p]]
starts = sorted(cst); ch = []
for ci, s0 in enumerate(starts):
    e0 = starts[ci+1] if ci + 1 < len(starts) else N
    ch.append([tok[p] for p in range(s0, e0) if not holes[p]])
while True:
    new = [greedy(c) for c in ch]
    ch = [x[0] for x in new]
    if sum(x[1] for x in new) == 0: break
flat = [t for c in ch for t in c]
print("tokens", len(flat), "expected", len(expt), "equal", flat == list(expt))
