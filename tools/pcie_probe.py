"""Host <-> device copy rates on the GPU box (informs the host-path pipeline design).

    python tools/pcie_probe.py
Pageable and pinned H2D / D2H of 256 MiB with torch, concurrent H2D + D2H on two streams, and
host memcpy bandwidth with 1..16 threads (numpy copies in a thread pool)."""
import json
import os
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch


def rate(f, nbytes, reps=5):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return round(nbytes * reps / (time.perf_counter() - t0) / 1e9, 2)


def main():
    n = 256 << 20
    res = {"host_cpus": os.cpu_count()}
    h = torch.empty(n, dtype=torch.uint8)
    h.numpy()[:] = 1
    hp = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
    res["h2d_pageable_GBps"] = rate(lambda: d.copy_(h), n)
    res["h2d_pinned_GBps"] = rate(lambda: d.copy_(hp, non_blocking=True), n)
    o = torch.empty(n, dtype=torch.uint8)
    op = torch.empty(n, dtype=torch.uint8).pin_memory()
    res["d2h_pageable_GBps"] = rate(lambda: o.copy_(d), n)
    res["d2h_pinned_GBps"] = rate(lambda: op.copy_(d, non_blocking=True), n)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def both():
        with torch.cuda.stream(s1):
            d2.copy_(hp, non_blocking=True)
        with torch.cuda.stream(s2):
            op.copy_(d, non_blocking=True)
    res["h2d_plus_d2h_pinned_GBps_each"] = rate(both, n)
    src = h.numpy()
    dst = np.empty(n, np.uint8)
    for k in (1, 2, 4, 8, 16):
        parts = np.array_split(np.arange(n), k)
        bounds = [(p[0], p[-1] + 1) for p in parts]
        with ThreadPoolExecutor(k) as ex:
            def cp():
                list(ex.map(lambda b: np.copyto(dst[b[0]:b[1]], src[b[0]:b[1]]), bounds))
            res[f"memcpy_{k}t_GBps"] = rate(cp, n)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
