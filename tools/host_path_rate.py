"""Rates that DESIGN.md quotes beside the bench line (one GPU).

    python tools/host_path_rate.py [--mib 1024]

1. cfg3 through the host-buffer entry point blt_bpe_process_chunks (pageable host input ->
   device -> host output, chunk lengths) at each --gpus n_gpus (device contexts; on a one-GPU box
   they share the device), with and without the pinned staging ring (--pin): the PCIe-inclusive
   rate.  Never the bench value.
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
    ap.add_argument("--gpus", default="1,8", help="n_gpus values for blt_bpe_process_chunks (contexts; on a one-GPU "
                                                   "box they share the device)")
    ap.add_argument("--no-cfg2", action="store_true")
    ap.add_argument("--pin", default="0,1", help="pinned staging ring off/on (blt_debug_set_pin_ring)")
    a = ap.parse_args()
    import blt_amd
    from blt_amd import synth
    from oracle import oracle as O

    res = {}
    n = a.mib << 20
    m3 = synth.merges_dict(synth.text_merges_50k(synth.text(64 << 20, seed=3), seed=3))
    s3 = blt_amd.BpeStrategy(m3)
    text = synth.text(n, seed=3)
    exp = O.COracle(m3).run(text, CHUNK, threads=16)
    import ctypes
    from blt_amd import _lib
    L = _lib.lib()
    out = np.empty(2 * n, np.uint8)   # one caller buffer, first-touched by the warm call
    olen = ctypes.c_size_t(0)
    runs = [(int(x), False) for x in a.gpus.split(",")]
    runs += [(g, True) for g, _ in runs if g > 1]   # n_gpus contexts sharing the one device
    runs = [(g, shared, int(p)) for g, shared in runs for p in a.pin.split(",")]
    for g, shared, pin in runs:
        L.blt_debug_set_shared_contexts(1 if shared else 0)
        L.blt_debug_set_pin_ring(pin)

        def call():
            _lib.check(L.blt_bpe_process_chunks(s3.handle, text.ctypes.data, n, CHUNK, g, out.ctypes.data, out.size,
                                                ctypes.byref(olen), None))
        call()       # device tables, context buffers
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            call()
            ts.append(time.perf_counter() - t0)
        dt = min(ts)
        L.blt_debug_set_shared_contexts(0)
        L.blt_debug_set_pin_ring(0)
        res[f"cfg3_host_path_n_gpus{g}" + ("_shared_contexts" if shared else "") + ("_pinned_ring" if pin else "")] = {
                                            "bytes": n, "n_gpus": g, "contexts": g if shared else 1,
                                            "pinned_ring": bool(pin),
                                            "seconds": round(dt, 4),
                                            "seconds_all": [round(t, 4) for t in ts],
                                            "GBps": round(n / dt / 1e9, 3),
                                            "bit_exact": bool(np.array_equal(out[:olen.value], exp))}
    if a.no_cfg2:
        print(json.dumps(res))
        return

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
