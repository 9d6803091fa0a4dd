"""Device-resident rates of every BASELINE config and §8 row beside the bench line (one GPU).

    python tools/config_rates.py [--mib 1024] [--only cfg2,cfg5,...]

Rows (inputs resident in HBM, kernel time from HIP events on the launch stream, median of
10 launches; every output checked bit-exactly against the C oracle or numpy):
  cfg2   100 MiB synthetic text, 256 merges ranked from it, 16 MiB chunks
  cfg3   the bench workload (1 GiB text, 50k merges)
  cfg5   random bytes (seed 5), cfg3's 50k merges, 16 MiB chunks (per-GPU share of config 5)
  basic  BasicTokenizationStrategy (f3): byte -> BE [0, b], 1 GiB random bytes
  multi  a general map that needs several passes (f2): chained and byte-valued merges on text
  host   cfg3 through blt_bpe_process_chunks from pageable host memory (PCIe-inclusive)
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHUNK = 16 << 20


def device_rate(strategy, host, cs, reps=10):
    import torch
    n = host.size
    d_in = torch.from_numpy(host).cuda()
    d_out = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
    wsb = strategy.workspace_size(n, cs)
    ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    tok = strategy.encode_device(d_in.data_ptr(), n, cs, d_out.data_ptr(), ws.data_ptr(), wsb, sp, sync=True)
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        strategy.encode_device(d_in.data_ptr(), n, cs, d_out.data_ptr(), ws.data_ptr(), wsb, sp, sync=False)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    strategy.check_workspace(ws.data_ptr(), sp)
    return float(np.median(ts)), tok, d_out[:2 * tok].cpu().numpy()


def row(n, ms, tok, exact, **kw):
    r = {"bytes": n, "ms": round(ms, 4), "input_GBps": round(n / ms / 1e6, 2), "tokens_per_byte": round(tok / n, 4),
         "algorithmic_GBps": round((n + 2 * tok) / ms / 1e6, 2),
         "hbm_frac": round((n + 2 * tok) / ms / 1e6 / 8000.0, 4), "bit_exact": exact}
    r.update(kw)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--only", default="cfg2,cfg3,cfg5,basic,multi,host")
    a = ap.parse_args()
    import torch
    import blt_amd
    from blt_amd import synth
    from oracle import oracle as O

    only = set(a.only.split(","))
    n = a.mib << 20
    res = {}
    m3 = synth.merges_dict(synth.text_merges_50k(synth.text(64 << 20, seed=3), seed=3))
    s3 = blt_amd.BpeStrategy(m3)
    if "cfg2" in only:
        t2 = synth.text(100 << 20, seed=2)
        m2 = synth.merges_dict(synth.top_pair_merges(t2, 256))
        s2 = blt_amd.BpeStrategy(m2)
        ms, tok, got = device_rate(s2, t2, CHUNK)
        res["cfg2"] = row(t2.size, ms, tok, bool(np.array_equal(got, O.COracle(m2).run(t2, CHUNK, threads=16))))
    if "cfg3" in only:
        t3 = synth.text(n, seed=3)
        ms, tok, got = device_rate(s3, t3, CHUNK)
        res["cfg3"] = row(n, ms, tok, bool(np.array_equal(got, O.COracle(m3).run(t3, CHUNK, threads=16))))
    if "cfg5" in only:
        r5 = synth.random_bytes(n, seed=5)
        ms, tok, got = device_rate(s3, r5, CHUNK)
        res["cfg5"] = row(n, ms, tok, bool(np.array_equal(got, O.COracle(m3).run(r5, CHUNK, threads=16))))
    if "basic" in only:
        rb = synth.random_bytes(n, seed=1)
        d_in = torch.from_numpy(rb).cuda()
        d_out = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
        bs = blt_amd.BasicTokenizationStrategy()
        sp = torch.cuda.current_stream().cuda_stream
        bs.encode_device(d_in.data_ptr(), n, d_out.data_ptr(), sp)
        ts = []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            bs.encode_device(d_in.data_ptr(), n, d_out.data_ptr(), sp)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        got = d_out.cpu().numpy()
        exp = np.zeros(2 * n, np.uint8)
        exp[1::2] = rb
        res["basic"] = row(n, float(np.median(ts)), n, bool(np.array_equal(got, exp)))
    if "multi" in only:
        tm = synth.text(256 << 20, seed=2)
        mm = {(101, 32): 256, (256, 116): 257, (116, 104): 65, (65, 101): 258, (32, 116): 259, (259, 104): 260}
        sm = blt_amd.BpeStrategy(mm)
        ms, tok, got = device_rate(sm, tm, CHUNK)
        res["multi"] = row(tm.size, ms, tok, bool(np.array_equal(got, O.COracle(mm).run(tm, CHUNK, threads=16))),
                           passes="general map (chained and byte-valued merges)")
    if "host" in only:
        # blt_bpe_process_chunks from pageable host memory into a caller buffer: the first call pays
        # device allocations and first-touch page faults of the output; steady state reuses both
        t3 = synth.text(n, seed=3)
        lib, h = blt_amd._lib.lib(), s3.handle
        out = np.empty(2 * n, np.uint8)
        olen = ctypes.c_size_t(0)

        def call():
            blt_amd._lib.check(lib.blt_bpe_process_chunks(h, t3.ctypes.data, n, CHUNK, 1, out.ctypes.data, out.size,
                                                          ctypes.byref(olen), None))
        t0 = time.perf_counter()
        call()
        cold = time.perf_counter() - t0
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            call()
            ts.append(time.perf_counter() - t0)
        dt = float(np.median(ts))
        exp = O.COracle(m3).run(t3, CHUNK, threads=16)
        res["host"] = {"bytes": n, "seconds": round(dt, 4), "input_GBps": round(n / dt / 1e9, 3),
                       "cold_seconds": round(cold, 4),
                       "bit_exact": bool(np.array_equal(out[:olen.value], exp))}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
