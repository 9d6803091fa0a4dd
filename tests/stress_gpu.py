"""Bounded randomized GPU stress run: many launch shapes in one process, each checked bit-exact
against the C oracle; device-side range/prefix checks surface as BltError with diagnostics.

    python tests/stress_gpu.py [seconds]
"""
import os
import random
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import blt_amd  # noqa: E402
from oracle import oracle as O  # noqa: E402


def rand_map(rng, alphabet):
    d = rng.choice([0.01, 0.2, 0.6, 1.0])
    keys = {(rng.randrange(alphabet), rng.randrange(alphabet)) for _ in range(int(d * alphabet * alphabet) + 1)}
    return {k: 256 + i for i, k in enumerate(sorted(keys))}


def main(seconds):
    rng = random.Random(12345)
    t0 = time.time()
    it = 0
    fails = 0
    while time.time() - t0 < seconds:
        it += 1
        alphabet = rng.choice([2, 4, 30, 256])
        m = rand_map(rng, alphabet)
        n = rng.choice([rng.randrange(1, 5000), rng.randrange(1, 200000), rng.randrange(200000, 3000000)])
        data = np.frombuffer(bytes(rng.randrange(alphabet) for _ in range(min(n, 4096))) * (n // 4096 + 1),
                             np.uint8)[:n].copy()
        cs = rng.choice([n, 262144, 300007, 1 << 20])
        s = blt_amd.BpeStrategy(m)
        try:
            if cs >= n:
                got = np.frombuffer(s.process_chunk(data), np.uint8)
            else:
                got = s.process_chunks(data, cs)
        except blt_amd.BltError as e:
            print(f"iter {it}: n={n} cs={cs} alphabet={alphabet} ERROR {e}", flush=True)
            fails += 1
            continue
        exp = O.COracle(m).run(data, max(cs, 1), threads=8) if cs < n else np.frombuffer(
            O.COracle(m).process_chunk(data), np.uint8)
        if not np.array_equal(got, exp):
            print(f"iter {it}: n={n} cs={cs} alphabet={alphabet} MISMATCH {got.size} vs {exp.size}", flush=True)
            fails += 1
        if it % 25 == 0:
            print(f"{it} iterations, {fails} failures, {time.time() - t0:.0f}s", flush=True)
    print(f"done: {it} iterations, {fails} failures")
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main(float(sys.argv[1]) if len(sys.argv) > 1 else 60))
