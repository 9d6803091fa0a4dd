"""One f2 row of bench.py's `configs` (a general map, device-resident), called --reps times
in one mode (asynchronous by default, as the row's `ms`): the program tools/pmc_profile.py profiles for a row's
HBM traffic per call (every kernel of the call: byte pass, chunk maps, u16 passes, chain end).

    python tools/f2_row.py --row chain|selfval|wrap|multi [--reps 5] [--sync]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--row", required=True)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sync", action="store_true", help="the calls ask for the token count (fused passes 1+2)")
    a = ap.parse_args()
    import torch
    import bench
    from blt_amd import synth
    host, make, _, desc = bench.general_workload(synth, a.row)
    n = host.size
    s = make()
    d_in = torch.from_numpy(host).cuda()
    d_out = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
    wsb = s.workspace_size(n, bench.CHUNK)
    ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    args = (d_in.data_ptr(), n, bench.CHUNK, d_out.data_ptr(), ws.data_ptr(), wsb, sp)
    for _ in range(a.reps):
        s.encode_device(*args, sync=a.sync)
    torch.cuda.synchronize()
    s.check_workspace(ws.data_ptr(), sp)
    print(f"{a.row}: {desc}; {n} bytes; {a.reps} {'synchronous' if a.sync else 'asynchronous'} calls")


if __name__ == "__main__":
    main()
