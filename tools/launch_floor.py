"""The floor of a HIP-event-timed launch on this box: events around a near-empty kernel
(torch.cuda._sleep of 1 cycle), median of 50, and around the byte-pass kernel on 1 MiB."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=50):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1000.0)
    return float(np.median(ts)), float(np.min(ts))


def main():
    torch.cuda.init()
    x = torch.zeros(1, device="cuda")
    res = {"sleep1_us": timed(lambda: torch.cuda._sleep(1)), "fill1_us": timed(lambda: x.fill_(1.0))}
    import blt_amd
    from blt_amd import synth
    text = synth.text(1 << 20, seed=2)
    m = synth.merges_dict(synth.top_pair_merges(synth.text(100 << 20, seed=2), 256))
    s = blt_amd.BpeStrategy(m)
    n = text.size
    d_in = torch.from_numpy(text).cuda()
    d_out = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
    wsb = s.workspace_size(n, 16 << 20)
    ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    s.encode_device(d_in.data_ptr(), n, 16 << 20, d_out.data_ptr(), ws.data_ptr(), wsb, sp, sync=True)

    def one():
        s.workspace_reset(ws.data_ptr(), n, 16 << 20, sp)
    res["workspace_reset_us"] = timed(one)

    def k():
        s.encode_device_prezeroed(d_in.data_ptr(), n, 16 << 20, d_out.data_ptr(), ws.data_ptr(), wsb, sp)
    ts = []
    for _ in range(50):
        one()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        k()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1000.0)
    res["scan_bytes_1MiB_us"] = (float(np.median(ts)), float(np.min(ts)))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
