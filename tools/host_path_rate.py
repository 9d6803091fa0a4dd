"""Rates that DESIGN.md quotes beside the bench line (one GPU).

    python tools/host_path_rate.py [--mib 1024]

1. cfg3 through the host-buffer entry point blt_bpe_process_chunks (pageable host input ->
   device -> host output, chunk lengths): the PCIe-inclusive rate.  Never the bench value.
2. cfg2 (256 merges, 100 MiB text, 16 MiB chunks) on device-resident buffers: kernel rate and
   output tokens per input byte.
Both outputs are checked bit-exactly against the C oracle.
"""
import argparse
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
        strategy.workspace_reset(ws.data_ptr(), n, cs, sp)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        strategy.encode_device_prezeroed(d_in.data_ptr(), n, cs, d_out.data_ptr(), ws.data_ptr(), wsb, sp)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    strategy.check_workspace(ws.data_ptr(), sp)
    return float(np.median(ts)), tok, d_out[:2 * tok].cpu().numpy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    a = ap.parse_args()
    import blt_amd
    from blt_amd import synth
    from oracle import oracle as O

    res = {}
    n = a.mib << 20
    m3 = synth.merges_dict(synth.text_merges_50k(synth.text(64 << 20, seed=3), seed=3))
    s3 = blt_amd.BpeStrategy(m3)
    text = synth.text(n, seed=3)
    s3.process_chunks(text[:1 << 20], CHUNK)       # warm the device tables
    t0 = time.perf_counter()
    out = s3.process_chunks(text, CHUNK)
    dt = time.perf_counter() - t0
    exp = O.COracle(m3).run(text, CHUNK, threads=16)
    res["cfg3_host_path"] = {"bytes": n, "seconds": round(dt, 4), "GBps": round(n / dt / 1e9, 3),
                             "bit_exact": bool(np.array_equal(out, exp))}

    t2 = synth.text(100 << 20, seed=2)
    m2 = synth.merges_dict(synth.top_pair_merges(t2, 256))
    s2 = blt_amd.BpeStrategy(m2)
    ms, tok, got = device_rate(s2, t2, CHUNK)
    exp2 = O.COracle(m2).run(t2, CHUNK, threads=16)
    res["cfg2_device"] = {"bytes": t2.size, "kernel_ms": round(ms, 4), "GBps": round(t2.size / ms / 1e6, 2),
                          "tokens_per_byte": round(tok / t2.size, 4),
                          "algorithmic_GBps": round((t2.size + 2 * tok) / ms / 1e6, 2),
                          "bit_exact": bool(np.array_equal(got, exp2))}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
