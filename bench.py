"""Benchmark of the BPE merge scan (BASELINE.json metric: input GB/s tokenized, % HBM roofline).

Workload (per GPU): BASELINE config 3 — 1 GiB of seeded synthetic English-like text, the
50 000-line merges built from that text (every pair seen, by frequency, then a seeded
permutation of the rest), --chunksize 16MB.  One step = one whole-buffer merge pass over the
rank's 1 GiB, inputs resident in HBM.  With N GPUs each rank tokenises its own 1 GiB shard of
an N GiB stream (config 4's sharding; chunks are independent, so no collective on the data
path) and `value` is the aggregate input rate: N x 1 GiB / max-over-ranks step time.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

Prints ONE JSON line on rank 0.  `roofline` prices the merge-scan kernel alone (HIP events on
its stream around each launch) against HBM: algorithmic bytes = input bytes + 2 x output
tokens.  `cpu_baseline` times the C restatement of the reference (hash-map, multi-pass,
task-per-chunk) on the same 1 GiB with one thread per usable host core (num_cpus semantics: the
cgroup quota, else the affinity mask; both counts are reported), and its output doubles as the
bit-exact check of the GPU output; `cpu_baseline_optimized` times a dense-table single-pass CPU
version beside it.

At N = 1 the line also carries (rank 0, outside the timed region of `value`):
  * `configs`: the other BASELINE workloads on the same kernel, device-resident, kernel-only
    (median of HIP-event timings), each with its roofline fraction and a bit-exact check:
    cfg2 (100 MiB text, 256 merges) and cfg5 (1 GiB random bytes, cfg3's 50k merges); `multi`:
    the f2 general map (256 MiB text, chained merges: one byte pass and u16 passes);
  * `end_to_end`: cfg3 through blt_bpe_process_chunks from pageable host memory (PCIe-inclusive);
  * `per_chunk_path`: 16 host threads calling blt_bpe_process_chunk on the 64 16-MiB chunks of
    cfg3 (the reference's per-chunk strategy calls, pipeline.rs:86, :141-150).
--workload cfg2|cfg5 makes that workload the timed one (for per-workload rocprofv3 runs).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = 1 << 30
CHUNK = 16 << 20
MERGES_SAMPLE = 64 << 20
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "input GB/s tokenized (BPE) at 1/2/4/8 MI355X; % HBM roofline"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bytes-per-gpu", type=int, default=GIB)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip configs / end_to_end / per_chunk_path")
    ap.add_argument("--workload", default="cfg3", choices=["cfg2", "cfg3", "cfg5"])
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("BLT_CPU_THREADS", "0")),
                    help="0: every usable host core (num_cpus semantics)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per launch (from tools/pmc_profile.py runs)")
    return ap.parse_args()


def usable_cores():
    """num_cpus::get() as the reference's tokio runtime sizes itself (src/main.rs:81): the cgroup
    CPU quota if set, else the affinity mask (blt_determine_thread_count(0, 0) computes it the
    same way); returns (usable, affinity, os.cpu_count())."""
    from blt_amd import _lib
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return int(_lib.lib().blt_determine_thread_count(0, 0)), aff, os.cpu_count() or 1


def kernel_ms(strategy, d_in, n, d_out, reps=20, warmup=5):
    """Median kernel time (HIP events on the launch stream, workspace reset outside them), after
    `warmup` untimed launches, the launches back to back: as the timed loop of `value`."""
    import torch
    wsb = strategy.workspace_size(n, CHUNK)
    ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    tok = strategy.encode_device(d_in.data_ptr(), n, CHUNK, d_out.data_ptr(), ws.data_ptr(), wsb, sp, sync=True)
    for _ in range(warmup):
        strategy.workspace_reset(ws.data_ptr(), n, CHUNK, sp)
        strategy.encode_device_prezeroed(d_in.data_ptr(), n, CHUNK, d_out.data_ptr(), ws.data_ptr(), wsb, sp)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in evs:
        strategy.workspace_reset(ws.data_ptr(), n, CHUNK, sp)
        e0.record(stream)
        strategy.encode_device_prezeroed(d_in.data_ptr(), n, CHUNK, d_out.data_ptr(), ws.data_ptr(), wsb, sp)
        e1.record(stream)
    torch.cuda.synchronize()
    strategy.check_workspace(ws.data_ptr(), sp)
    return float(np.median([e0.elapsed_time(e1) for e0, e1 in evs])), tok


def workload(synth, name, n):
    """(host bytes, merges, description) of a BASELINE workload."""
    if name == "cfg2":
        host = synth.text(100 << 20, seed=2)
        return host, synth.merges_dict(synth.top_pair_merges(host, 256)), \
            "cfg2: 100 MiB synthetic text, 256 merges ranked from it, --chunksize 16MB"
    merges = build_merges(synth)
    if name == "cfg5":
        return synth.random_bytes(n, seed=5), merges, \
            f"cfg5 (per-GPU share): {n >> 20} MiB random bytes, cfg3's 50000-line merges, --chunksize 16MB"
    return None, merges, f"cfg3: {n >> 30} GiB synthetic text per GPU, 50000-line merges, --chunksize 16MB"


def extra_configs(blt_amd, synth, O, threads):
    """cfg2 and cfg5 on the same kernel (kernel-only rates, bit-exact against the oracle)."""
    import torch
    res = {}
    for name in ("cfg2", "cfg5"):
        host, merges, desc = workload(synth, name, GIB)
        s = blt_amd.BpeStrategy(merges)
        n = host.size
        d_in = torch.from_numpy(host).cuda()
        d_out = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
        ms, tok = kernel_ms(s, d_in, n, d_out)
        got = d_out[:2 * tok].cpu().numpy()
        exp = O.COracle(merges).run(host, CHUNK, threads=threads)
        algo = n + 2 * tok
        res[name] = {"workload": desc, "bytes": n, "kernel_ms": round(ms, 4),
                     "input_GBps": round(n / ms / 1e6, 1), "achieved_GBps": round(algo / ms / 1e6, 1),
                     "frac": round(algo / ms / 1e6 / HBM_PEAK_GBS, 4), "tokens_per_byte": round(tok / n, 4),
                     "bit_exact_vs_oracle": bool(exp.size == got.size and np.array_equal(exp, got))}
        del d_in, d_out
        s.close()
    res["multi"] = general_map_rate(blt_amd, synth, O, threads)
    return res


# f2: a general map that needs more than one pass (chained and byte-valued merges, SURVEY.md §8a
# row f2): one byte pass, then u16 passes until the chain provably stops.
MULTI_MAP = {(101, 32): 256, (256, 116): 257, (116, 104): 65, (65, 101): 258, (32, 116): 259, (259, 104): 260}


def general_map_rate(blt_amd, synth, O, threads, reps=10):
    """256 MiB of cfg2's text through the chained map, device-resident; the timed region is the
    whole encode_device call (byte pass, u16 passes, the host's read of the pass count)."""
    import torch
    host = synth.text(256 << 20, seed=2)
    n = host.size
    s = blt_amd.BpeStrategy(MULTI_MAP)
    d_in = torch.from_numpy(host).cuda()
    d_out = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
    wsb = s.workspace_size(n, CHUNK)
    ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    tok = s.encode_device(d_in.data_ptr(), n, CHUNK, d_out.data_ptr(), ws.data_ptr(), wsb, sp, sync=True)
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        s.encode_device(d_in.data_ptr(), n, CHUNK, d_out.data_ptr(), ws.data_ptr(), wsb, sp, sync=False)
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = float(np.median(ts))
    passes = int(blt_amd._lib.lib().blt_debug_last_u16_passes())
    got = d_out[:2 * tok].cpu().numpy()
    exp = O.COracle(MULTI_MAP).run(host, CHUNK, threads=threads)
    algo = n + 2 * tok
    s.close()
    return {"workload": "f2: 256 MiB synthetic text (cfg2's), chained + byte-valued 6-entry map, --chunksize 16MB",
            "bytes": n, "ms": round(ms, 4), "u16_passes": passes, "input_GBps": round(n / ms / 1e6, 1),
            "achieved_GBps": round(algo / ms / 1e6, 1), "frac": round(algo / ms / 1e6 / HBM_PEAK_GBS, 4),
            "tokens_per_byte": round(tok / n, 4),
            "bit_exact_vs_oracle": bool(exp.size == got.size and np.array_equal(exp, got))}


def host_paths(blt_amd, strategy, host, exp):
    """PCIe-inclusive rates of the host-buffer entry points on the cfg3 bytes (never `value`)."""
    import ctypes
    import threading
    from blt_amd import _lib
    L, h, n = _lib.lib(), strategy.handle, host.size
    out = np.empty(2 * n, np.uint8)
    olen = ctypes.c_size_t(0)
    ts = []
    for _ in range(4):   # the first call pays device allocations and first-touch faults
        t0 = time.perf_counter()
        _lib.check(L.blt_bpe_process_chunks(h, host.ctypes.data, n, CHUNK, 1, out.ctypes.data, out.size,
                                            ctypes.byref(olen), None))
        ts.append(time.perf_counter() - t0)
    e2e = {"value": round(n / min(ts[1:]) / 1e9, 3), "unit": "GB/s", "cold_seconds": round(ts[0], 4),
           "path": "blt_bpe_process_chunks, pageable host in/out, 1 GPU (H2D + kernel + D2H pipelined)",
           "bit_exact_vs_oracle": bool(np.array_equal(out[:olen.value], exp))}
    # per-chunk trait path: 16 threads, one process_chunk per 16 MiB chunk
    nch = n // CHUNK
    outs = [np.empty(2 * CHUNK, np.uint8) for _ in range(16)]
    lens = [0] * nch
    errs = []

    def worker(t):
        ol = ctypes.c_size_t(0)
        for k in range(t, nch, 16):
            rc = L.blt_bpe_process_chunk(h, host.ctypes.data + k * CHUNK, CHUNK, outs[t].ctypes.data, 2 * CHUNK,
                                         ctypes.byref(ol))
            if rc:
                errs.append(rc)
            lens[k] = ol.value
    best = None
    for _ in range(3):
        th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    per = {"value": round(nch * CHUNK / best / 1e9, 3), "unit": "GB/s", "threads": 16, "chunk_bytes": CHUNK,
           "chunks": nch, "path": "blt_bpe_process_chunk per 16 MiB chunk from 16 host threads (pageable)",
           "errors": len(errs), "bytes_match_batched": bool(sum(lens) == olen.value)}
    return e2e, per


def build_merges(synth):
    """cfg3 merges: ranked pairs of the first 64 MiB of the seed-3 text, then a seeded
    permutation of the unseen pairs, 50 000 lines."""
    sample = synth.text(MERGES_SAMPLE, seed=3, offset=0)
    return synth.merges_dict(synth.text_merges_50k(sample, seed=3))


def relaunch(n):
    """`python bench.py --gpus N` outside a launcher: start one process per GPU under
    torch.distributed.run as a child (nothing here has touched the GPU) and return its exit code."""
    import subprocess
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch(args.gpus))
    import torch
    import torch.distributed as dist

    import blt_amd
    from blt_amd import shard, synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    # BLT_BENCH_BACKEND=gloo with BLT_BENCH_DEVICE=0 rehearses the N > 1 path with every rank on one
    # GPU (RCCL refuses two ranks on one device); the driver's runs use RCCL, one GPU per rank
    backend = os.environ.get("BLT_BENCH_BACKEND", "nccl")
    dev = int(os.environ.get("BLT_BENCH_DEVICE", local))
    torch.cuda.set_device(dev)
    if distributed:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)

    n = args.bytes_per_gpu
    wl_host, merges, wl_desc = workload(synth, args.workload, n)
    strategy = blt_amd.BpeStrategy(merges)
    if wl_host is None:
        b0, b1 = shard.rank_bytes(world * n, CHUNK, rank, world)   # this rank's chunk range of the stream
        host = synth.text(b1 - b0, seed=3, offset=b0)
    else:
        host = wl_host
        n = host.size
    d_in = torch.from_numpy(host).to("cuda")
    d_out = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
    nchunks = (n + CHUNK - 1) // CHUNK
    d_off = torch.zeros(nchunks + 1, dtype=torch.int64, device="cuda")
    wsb = strategy.workspace_size(n, CHUNK)
    ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    args_dev = (d_in.data_ptr(), n, CHUNK, d_out.data_ptr(), ws.data_ptr(), wsb, sp, d_off.data_ptr())

    def step(ev0=None, ev1=None):
        strategy.workspace_reset(ws.data_ptr(), n, CHUNK, sp)
        if ev0 is not None:
            ev0.record(stream)
        strategy.encode_device_prezeroed(*args_dev)
        if ev1 is not None:
            ev1.record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    strategy.check_workspace(ws.data_ptr(), sp)

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(*evs[i])
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    strategy.check_workspace(ws.data_ptr(), sp)
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    tokens = int(d_off[-1].item())

    elapsed, kern_ms_max = shard.max_over_ranks([elapsed, kern_ms], device="cuda" if backend == "nccl" else None)
    ms_per_step = 1000.0 * elapsed / args.steps
    value = world * n / (elapsed / args.steps) / 1e9

    algo_bytes = n + 2 * tokens                               # N + 2M per launch
    achieved = algo_bytes / (kern_ms / 1000.0) / 1e9
    traffic = None
    if os.path.exists(args.traffic):
        with open(args.traffic) as f:
            tj = json.load(f)
        tw = tj.get("workloads", {}).get(args.workload, {})
        if tw.get("bytes_per_gpu") == n and tw.get("chunk_size") == CHUNK:
            traffic = tw.get("hbm_bytes_per_launch")

    cpu = None
    cpu_opt = None
    exact = None
    usable, affinity, ncpu = usable_cores()
    threads = max(1, args.cpu_threads or usable)
    extras = {}
    if rank == 0 and not args.no_cpu_baseline and distributed:
        # N > 1: the CPU baseline is reported at N = 1 only; rank 0 still checks its shard
        # bit-exact, with the dense single-pass oracle (outside the timed region)
        from oracle import oracle as O
        fast = O.fast_run(merges, host, CHUNK, threads=threads)
        if fast is not None:
            exact = bool(np.array_equal(fast, d_out[:2 * tokens].cpu().numpy()))
    elif rank == 0 and not args.no_cpu_baseline:
        from oracle import oracle as O
        orc = O.COracle(merges)
        c0 = time.perf_counter()
        exp = orc.run(host, CHUNK, threads=threads)
        cpu_s = time.perf_counter() - c0
        cpu = {"value": round(n / cpu_s / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port",
               "usable_cores": usable, "affinity_cpus": affinity, "os_cpu_count": ncpu,
               "sample": f"the same {n >> 20} MiB {args.workload} shard, {nchunks} chunks of 16 MiB, C restatement "
                         f"of tokenizer.rs:56-93 (hash map, multi-pass), one task per chunk on {threads} threads "
                         f"(every usable core: cgroup quota, else affinity mask, as num_cpus)",
               "seconds": round(cpu_s, 3)}
        got = d_out[:2 * tokens].cpu().numpy()
        exact = bool(exp.size == got.size and np.array_equal(exp, got))
        # SURVEY.md §8(d)'s "optimised CPU" line beside it: dense table, one greedy pass per chunk
        c0 = time.perf_counter()
        fast = O.fast_run(merges, host, CHUNK, threads=threads)
        fast_s = time.perf_counter() - c0
        if fast is not None:
            cpu_opt = {"value": round(n / fast_s / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port-optimized",
                       "sample": f"the same {n >> 20} MiB {args.workload} shard: dense 64K-entry table, one greedy "
                                 f"pass per chunk (single-pass map), {threads} threads", "seconds": round(fast_s, 3),
                       "matches_port": bool(np.array_equal(fast, exp))}
        if not args.no_extra and args.workload == "cfg3":
            del d_in, d_out, ws
            extras["configs"] = extra_configs(blt_amd, synth, O, threads)
            extras["end_to_end"], extras["per_chunk_path"] = host_paths(blt_amd, strategy, host, exp)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": ("synthetic: seeded uniform random bytes (splitmix64), cfg3's merges" if args.workload == "cfg5" else
                     "synthetic: seeded English-like text (splitmix64, 1 MiB blocks), merges ranked from it"),
            "config": {"workload": wl_desc,
                       "bytes_per_gpu": n, "chunk_size": CHUNK, "merges": len(merges),
                       "parallelism": f"chunk-sharded x{world}, no collective"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": "seg::scan_bytes_kernel<true, true>", "kernel_ms": round(kern_ms, 4),
                         "kernel_ms_max_rank": round(kern_ms_max, 4),
                         "algorithmic_bytes_per_launch": algo_bytes},
            "cpu_baseline": cpu,
            "cpu_baseline_optimized": cpu_opt,
            "bit_exact_vs_oracle": exact,
            "output_tokens_per_gpu": tokens,
        }
        line.update(extras)
        print(json.dumps(line), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
