"""Kernel-only timing of the byte-pass merge scan on cfg2 / cfg3 / cfg5 (one GPU, one library build).

    BLT_LIB_PATH=build/xp/libblt_bpe_X.so python tools/kbench.py [--only cfg3,cfg5] [--check]

Inputs resident in HBM; per config the median of --reps launches timed with HIP events on the
launch stream, the workspace reset outside the events.  --check compares the output with the
dense single-pass oracle (test infrastructure only).  Prints one JSON line per config.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHUNK = 16 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="cfg2,cfg3,cfg5")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("BLT_LIB_PATH", "product")))
    a = ap.parse_args()
    import torch
    import blt_amd
    from blt_amd import synth

    n = a.mib << 20
    m3 = synth.merges_dict(synth.text_merges_50k(synth.text(64 << 20, seed=3), seed=3))
    for cfg in a.only.split(","):
        if cfg == "cfg2":
            host = synth.text(100 << 20, seed=2)
            merges = synth.merges_dict(synth.top_pair_merges(host, 256))
        elif cfg == "cfg3":
            host, merges = synth.text(n, seed=3), m3
        elif cfg == "cfg5":
            host, merges = synth.random_bytes(n, seed=5), m3
        elif cfg.startswith("text"):   # textN: N MiB of cfg2's text with cfg2's merges (size sweeps)
            mib = int(cfg[4:])
            host = synth.text(mib << 20, seed=2)
            merges = synth.merges_dict(synth.top_pair_merges(synth.text(100 << 20, seed=2), 256))
        elif cfg == "same":   # --mib of one repeated byte under cfg3's merges: dense, every lookup one LDS entry
            host, merges = np.full(n, 101, np.uint8), m3
        elif cfg == "cfg2big":   # cfg2's text and merges at the --mib size: steady-state cost per tile
            host = synth.text(n, seed=2)
            merges = synth.merges_dict(synth.top_pair_merges(host[: 100 << 20], 256))
        else:
            raise SystemExit(f"unknown config {cfg}")
        s = blt_amd.BpeStrategy(merges)
        nb = host.size
        d_in = torch.from_numpy(host).cuda()
        d_out = torch.empty(2 * nb, dtype=torch.uint8, device="cuda")
        wsb = s.workspace_size(nb, CHUNK)
        ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
        sp = torch.cuda.current_stream().cuda_stream
        tok = s.encode_device(d_in.data_ptr(), nb, CHUNK, d_out.data_ptr(), ws.data_ptr(), wsb, sp, sync=True)
        ts = []
        for _ in range(a.reps):
            s.workspace_reset(ws.data_ptr(), nb, CHUNK, sp)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            s.encode_device_prezeroed(d_in.data_ptr(), nb, CHUNK, d_out.data_ptr(), ws.data_ptr(), wsb, sp)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        err = None
        try:
            s.check_workspace(ws.data_ptr(), sp)
        except Exception as ex:  # timing variants may flag errors
            err = str(ex)[:80]
        ms = float(np.median(ts))
        r = {"tag": a.tag, "cfg": cfg, "ms": round(ms, 4), "min_ms": round(min(ts), 4),
             "frac": round((nb + 2 * tok) / ms / 1e6 / 8000.0, 4), "tokens_per_byte": round(tok / nb, 4)}
        if err:
            r["err"] = err
        if a.check:
            from oracle import oracle as O
            exp = O.fast_run(merges, host, CHUNK, threads=16)
            r["bit_exact"] = bool(exp is not None and np.array_equal(exp, d_out[:2 * tok].cpu().numpy()))
        print(json.dumps(r), flush=True)
        del d_in, d_out, ws


if __name__ == "__main__":
    main()
