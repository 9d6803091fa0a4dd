"""Debug aid: replays one stress-test input on the GPU and compares every tile's look-back status
word with a sequential scan.  python tests/debug_replay.py <stress-iteration> [repeats]

The per-tile records exist only in a record build of the kernels:
    tools/build_variant.sh record -DBLT_DEBUG_RECORD=1
    BLT_LIB_PATH=build/exp/libblt_bpe_record.so python tests/debug_replay.py N"""
import os
import random
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import blt_amd  # noqa: E402
from oracle import oracle as O  # noqa: E402

TILE = 32768


def rand_map(rng, alphabet):
    d = rng.choice([0.01, 0.2, 0.6, 1.0])
    keys = {(rng.randrange(alphabet), rng.randrange(alphabet)) for _ in range(int(d * alphabet * alphabet) + 1)}
    return {k: 256 + i for i, k in enumerate(sorted(keys))}


def replay(target):
    rng = random.Random(12345)
    for it in range(1, target + 1):
        alphabet = rng.choice([2, 4, 30, 256])
        m = rand_map(rng, alphabet)
        n = rng.choice([rng.randrange(1, 5000), rng.randrange(1, 200000), rng.randrange(200000, 3000000)])
        data = np.frombuffer(bytes(rng.randrange(alphabet) for _ in range(min(n, 4096))) * (n // 4096 + 1),
                             np.uint8)[:n].copy()
        cs = rng.choice([n, 262144, 300007, 1 << 20])
    return m, data, cs


def expected_tiles(m, data, cs):
    n = data.size
    d = data.tolist()
    L = 1
    cnt = 0
    tiles = []
    for i in range(n):
        if i % TILE == 0:
            tiles.append((L, cnt))
        mi = i + 1 < n and (i + 1) % cs != 0 and (d[i], d[i + 1]) in m
        if L:
            cnt += 1
        L = 0 if (L and mi) else 1
    tiles.append((L, cnt))
    return tiles  # tiles[T] = (carry into T, tokens before T)


def tile_fn(m, d, cs, T, c):
    n = len(d)
    L = c
    cnt = 0
    for i in range(T * TILE, min(n, (T + 1) * TILE)):
        mi = i + 1 < n and (i + 1) % cs != 0 and (d[i], d[i + 1]) in m
        if L:
            cnt += 1
        L = 0 if (L and mi) else 1
    return cnt, L


def main():
    target = int(sys.argv[1])
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    m, data, cs = replay(target)
    n = data.size
    exp = O.COracle(m).run(data, cs, threads=8)
    tiles = expected_tiles(m, data, cs)
    print(f"n={n} cs={cs} ntiles={(n + TILE - 1) // TILE} expected tokens={exp.size // 2} seq={tiles[-1][1]}")
    s = blt_amd.BpeStrategy(m)
    d_in = torch.from_numpy(data).cuda()
    d_out = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
    wsb = s.workspace_size(n, cs)
    ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    import ctypes
    ntiles = (n + TILE - 1) // TILE
    dbg = torch.zeros(4 * ntiles, dtype=torch.int64, device="cuda")
    L = blt_amd._lib.lib()
    L.blt_debug_set_tile_record.argtypes = [ctypes.c_void_p]
    L.blt_debug_set_tile_record(dbg.data_ptr())
    dl = data.tolist()
    for r in range(reps):
        try:
            tok = s.encode_device(d_in.data_ptr(), n, cs, d_out.data_ptr(), ws.data_ptr(), wsb, stream, sync=True)
        except blt_amd.BltError as e:
            print("rep", r, "error", e)
            continue
        got = d_out[:2 * tok].cpu().numpy()
        ok = tok * 2 == exp.size and np.array_equal(got, exp)
        st = ws[64:64 + 8 * ((n + TILE - 1) // TILE)].cpu().numpy().view(np.uint64)
        bad = []
        for T, w in enumerate(st):
            w = int(w)
            flag, carry, off = w >> 62, (w >> 61) & 1, w & ((1 << 61) - 1)
            ec, eo = tiles[T + 1]
            if flag != 2 or carry != ec or off != eo:
                bad.append((T, flag, carry, off, ec, eo))
        first_diff = None
        if not ok:
            k = min(got.size, exp.size)
            diff = np.nonzero(got[:k] != exp[:k])[0]
            first_diff = int(diff[0]) if diff.size else k
        print(f"rep {r}: tokens={tok} ok={ok} first_diff_byte={first_diff} bad_tiles={bad[:6]}")
        if bad and r == 0:
            rec = dbg.cpu().numpy().astype(np.uint64)
            for T in range(max(0, bad[0][0] - 2), min(ntiles, bad[0][0] + 2)):
                O_, ch, cn, co = (int(x) for x in rec[4 * T:4 * T + 4])
                print(f"  tile {T}: O={O_} C={ch >> 32} how={ch & 0xffffffff:#x} cnt0={cn & 0xffffffff} "
                      f"cnt1={cn >> 32} co0={co & 1} co1={co >> 32}  expected C={tiles[T][0]} O={tiles[T][1]} "
                      f"fn0={tile_fn(m, dl, cs, T, 0)} fn1={tile_fn(m, dl, cs, T, 1)}")


if __name__ == "__main__":
    main()
