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
task-per-chunk over all threads) on the same 1 GiB, and its output doubles as the bit-exact
check of the GPU output; `cpu_baseline_optimized` times a dense-table single-pass CPU version
beside it.
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
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("BLT_CPU_THREADS", "16")))
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per launch (tools/pmc_traffic.py output)")
    return ap.parse_args()


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
    merges = build_merges(synth)
    strategy = blt_amd.BpeStrategy(merges)
    b0, b1 = shard.rank_bytes(world * n, CHUNK, rank, world)   # this rank's chunk range of the stream
    host = synth.text(b1 - b0, seed=3, offset=b0)
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
        if tj.get("bytes_per_gpu") == n and tj.get("chunk_size") == CHUNK:
            traffic = tj.get("hbm_bytes_per_launch")

    cpu = None
    cpu_opt = None
    exact = None
    if rank == 0 and not args.no_cpu_baseline and distributed:
        # N > 1: the CPU baseline is reported at N = 1 only; rank 0 still checks its shard
        # bit-exact, with the dense single-pass oracle (outside the timed region)
        from oracle import oracle as O
        threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        fast = O.fast_run(merges, host, CHUNK, threads=threads)
        if fast is not None:
            exact = bool(np.array_equal(fast, d_out[:2 * tokens].cpu().numpy()))
    elif rank == 0 and not args.no_cpu_baseline:
        from oracle import oracle as O
        orc = O.COracle(merges)
        threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        c0 = time.perf_counter()
        exp = orc.run(host, CHUNK, threads=threads)
        cpu_s = time.perf_counter() - c0
        cpu = {"value": round(n / cpu_s / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port",
               "sample": f"the same {n >> 20} MiB cfg3 shard, {nchunks} chunks of 16 MiB, C restatement of "
                         f"tokenizer.rs:56-93 (hash map, multi-pass) on {threads} threads",
               "seconds": round(cpu_s, 3)}
        got = d_out[:2 * tokens].cpu().numpy()
        exact = bool(exp.size == got.size and np.array_equal(exp, got))
        # SURVEY.md §8(d)'s "optimised CPU" line beside it: dense table, one greedy pass per chunk
        c0 = time.perf_counter()
        fast = O.fast_run(merges, host, CHUNK, threads=threads)
        fast_s = time.perf_counter() - c0
        if fast is not None:
            cpu_opt = {"value": round(n / fast_s / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port-optimized",
                       "sample": f"the same {n >> 20} MiB cfg3 shard: dense 64K-entry table, one greedy pass per "
                                 f"chunk (single-pass map), {threads} threads", "seconds": round(fast_s, 3),
                       "matches_port": bool(np.array_equal(fast, exp))}

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: seeded English-like text (splitmix64, 1 MiB blocks), merges ranked from it",
            "config": {"workload": "cfg3: 1 GiB synthetic text per GPU, 50000-line merges, --chunksize 16MB",
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
        print(json.dumps(line), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
