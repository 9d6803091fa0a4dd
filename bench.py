"""Benchmark of the BPE merge scan (BASELINE.json metric: input GB/s tokenized, % HBM roofline).

Workloads (one step = one whole-buffer merge pass over each rank's shard, inputs
resident in HBM; chunks are independent, so ranks share nothing and no collective touches the data):
  cfg3 (default at N = 1): 1 GiB of seeded synthetic English-like text per GPU, the 50 000-line
       merges built from that text, --chunksize 16MB (weak scaling: 1 GiB per rank at any N);
  cfg4 (default at N > 1): ONE 8 GiB stream of the same text split over the N ranks by whole
       chunks (shard.rank_bytes: 4 / 2 / 1 GiB per rank at N = 2 / 4 / 8; strong scaling);
  cfg5: ONE 4 GiB stream of uniform random bytes, cfg3's merges, split the same way (strong);
  cfg2: 100 MiB of text with 256 merges ranked from it (one GPU).
--total-bytes overrides the stream size of cfg4 / cfg5.  `value` = bytes all ranks processed /
max-over-ranks step time; `config.rank_bytes` lists every rank's byte range of the stream.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg3|cfg4|cfg5|cfg2]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

Prints ONE JSON line on rank 0.  `roofline` prices the merge-scan kernel alone (HIP events on
its stream around each launch) against HBM: algorithmic bytes = input bytes + 2 x output
tokens; `traffic` is the PMC-measured HBM bytes per launch from profiles/traffic.json, used only
when that record names this workload, size and the sha256 of the kernel source it was measured
on (else null).  `cpu_baseline` times the C restatement of the reference (hash-map, multi-pass,
task-per-chunk) on rank 0's shard (N = 1 only) with one thread per usable host core (num_cpus
semantics: min(cgroup quota, affinity mask)); its output doubles as the bit-exact check of the
GPU output; `cpu_baseline_optimized` times a dense-table single-pass CPU version beside it.

At N = 1 with the cfg3 workload the line also carries (rank 0, outside the timed region):
  * `configs`: the other workloads device-resident, kernel-only (median of HIP-event timings),
    each with its roofline fraction and a bit-exact check: cfg2, cfg5 (the whole 4 GiB stream on
    one GPU), and the general maps of row f2 (the whole encode_device call: byte pass, u16 passes,
    the host's read of the pass count): `multi` (chained + byte-valued merges on text), `wrap`
    (the 65 537-line merges file whose ids wrap: the L2 bucket table), `selfval` (merges valued
    their own first byte: the generic byte pass), `chain` (a 24-level doubling chain: u16 passes
    down to the generic token pass);
  * `end_to_end`: cfg3 through blt_bpe_process_chunks from pageable host memory (PCIe-inclusive);
  * `per_chunk_path`: 16 host threads calling blt_bpe_process_chunk on the 64 16-MiB chunks;
  * `cli_end_to_end`: the `blt` command line on cfg3's 1 GiB as a file on tmpfs to a tmpfs
    output (the reference's only published figure is its binary's file rate, README.md:272-278).
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
    ap.add_argument("--bytes-per-gpu", type=int, default=GIB, help="cfg3's bytes per rank")
    ap.add_argument("--total-bytes", type=int, default=0, help="cfg4 / cfg5 stream size (default 8 GiB / 4 GiB)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip configs / end_to_end / per_chunk_path / cli")
    ap.add_argument("--only-configs", default="", help="comma list: run only these `configs` rows")
    ap.add_argument("--events-outside-timed-loop", action="store_true",
                    help="time the kernel's HIP events in a second loop instead of inside the timed region "
                         "(experiment: shows what the event records cost `value`)")
    ap.add_argument("--reset-each-step", action="store_true",
                    help="enqueue a workspace reset before every step (experiment: what the kernel's "
                         "self-reset saves `value`)")
    ap.add_argument("--workload", default="", choices=["", "cfg2", "cfg3", "cfg4", "cfg5"],
                    help="default: cfg3 at N = 1, cfg4 at N > 1")
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
    # the byte-scan kernel leaves its ticket and status words zeroed (self-reset): launches follow
    # each other without a reset between them
    for _ in range(warmup):
        strategy.encode_device_prezeroed(d_in.data_ptr(), n, CHUNK, d_out.data_ptr(), ws.data_ptr(), wsb, sp)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in evs:
        e0.record(stream)
        strategy.encode_device_prezeroed(d_in.data_ptr(), n, CHUNK, d_out.data_ptr(), ws.data_ptr(), wsb, sp)
        e1.record(stream)
    torch.cuda.synchronize()
    strategy.check_workspace(ws.data_ptr(), sp)
    return float(np.median([e0.elapsed_time(e1) for e0, e1 in evs])), tok


STRONG_TOTAL = {"cfg4": 8 * GIB, "cfg5": 4 * GIB}


def workload(synth, name, rank=0, world=1, per_gpu=GIB, total=0):
    """(host bytes of this rank's shard, merges, description, (b0, b1) of the stream, stream bytes)
    of a BASELINE workload."""
    if name == "cfg2":
        host = synth.text(100 << 20, seed=2)
        return host, synth.merges_dict(synth.top_pair_merges(host, 256)), \
            "cfg2: 100 MiB synthetic text, 256 merges ranked from it, --chunksize 16MB", (0, host.size), host.size
    merges = build_merges(synth)
    from blt_amd import shard
    if name == "cfg3":   # weak: 1 GiB per rank, rank r's slice of an N GiB stream
        stream = world * per_gpu
        b0, b1 = shard.rank_bytes(stream, CHUNK, rank, world)
        return synth.text(b1 - b0, seed=3, offset=b0), merges, \
            f"cfg3: {per_gpu >> 20} MiB synthetic text per GPU, 50000-line merges, --chunksize 16MB", (b0, b1), stream
    stream = total or STRONG_TOTAL[name]
    b0, b1 = shard.rank_bytes(stream, CHUNK, rank, world)
    if name == "cfg4":
        return synth.text(b1 - b0, seed=3, offset=b0), merges, \
            f"cfg4: one {stream >> 20} MiB synthetic-text stream split over {world} GPU(s), 50000-line merges, " \
            f"--chunksize 16MB", (b0, b1), stream
    return synth.random_bytes(b1 - b0, seed=5, offset=b0), merges, \
        f"cfg5: one {stream >> 20} MiB random-byte stream split over {world} GPU(s), cfg3's 50000-line merges, " \
        f"--chunksize 16MB, --type audio", (b0, b1), stream


def extra_configs(blt_amd, synth, O, threads, only=()):
    """cfg2, cfg5 and the f2 general maps (kernel-only rates, bit-exact against the oracle)."""
    import torch
    res = {}
    for name in ("cfg2", "cfg5"):
        if only and name not in only:
            continue
        host, merges, desc, _, _ = workload(synth, name)
        s = blt_amd.BpeStrategy(merges)
        n = host.size
        d_in = torch.from_numpy(host).cuda()
        d_out = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
        ms, tok = kernel_ms(s, d_in, n, d_out)
        got = d_out[:2 * tok].cpu().numpy()
        exp = O.COracle(merges).run(host, CHUNK, threads=threads)
        algo = n + 2 * tok
        res[name] = {"workload": desc + (" (the whole stream on one GPU)" if name == "cfg5" else ""), "bytes": n,
                     "kernel_ms": round(ms, 4), "input_GBps": round(n / ms / 1e6, 1),
                     "achieved_GBps": round(algo / ms / 1e6, 1), "frac": round(algo / ms / 1e6 / HBM_PEAK_GBS, 4),
                     "tokens_per_byte": round(tok / n, 4),
                     "bit_exact_vs_oracle": bool(exp.size == got.size and np.array_equal(exp, got))}
        del d_in, d_out, got, exp, host
        s.close()
    for name in ("multi", "wrap", "selfval", "chain", "cyclic_dense"):
        if only and name not in only:
            continue
        res[name] = general_map_rate(blt_amd, synth, O, threads, name)
    if not only or "basic" in only:
        res["basic"] = basic_rate(blt_amd, synth, O, threads)
    return res


def basic_rate(blt_amd, synth, O, threads, n=GIB, reps=20, warmup=5):
    """Row f3 / cfg1 at scale: the basic strategy (tokenizer.rs:108-124, byte b -> BE [0, b]) on
    1 GiB of seeded random bytes (cfg1's generator, seed 1), basic_expand_kernel device-resident,
    median of HIP-event timings; algorithmic bytes N + 2N; checked against the oracle."""
    import torch
    host = synth.random_bytes(n, seed=1)
    s = blt_amd.BasicTokenizationStrategy()
    d_in = torch.from_numpy(host).cuda()
    d_out = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    for _ in range(warmup):
        s.encode_device(d_in.data_ptr(), n, d_out.data_ptr(), sp)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in evs:
        e0.record(stream)
        s.encode_device(d_in.data_ptr(), n, d_out.data_ptr(), sp)
        e1.record(stream)
    torch.cuda.synchronize()
    ms = float(np.median([e0.elapsed_time(e1) for e0, e1 in evs]))
    got = d_out.cpu().numpy()
    exp = O.COracle(None).run(host, CHUNK, threads=threads)
    algo = 3 * n
    return {"workload": "cfg1 at scale: 1024 MiB seeded random bytes, basic strategy (no merges)", "bytes": n,
            "kernel": "basic_expand_kernel", "kernel_ms": round(ms, 4), "input_GBps": round(n / ms / 1e6, 1),
            "achieved_GBps": round(algo / ms / 1e6, 1), "frac": round(algo / ms / 1e6 / HBM_PEAK_GBS, 4),
            "bit_exact_vs_oracle": bool(exp.size == got.size and np.array_equal(exp, got))}


def general_workload(synth, name):
    """(host bytes, strategy factory, merges for the oracle, description) of an f2 workload."""
    import blt_amd
    if name == "multi":
        m = synth.CHAINED_TEXT_MAP
        return synth.text(256 << 20, seed=2), lambda: blt_amd.BpeStrategy(m), m, \
            "f2: 256 MiB synthetic text (cfg2's), chained + byte-valued 6-entry map, --chunksize 16MB"
    if name == "selfval":
        m = synth.SELF_VALUED_MAP
        return synth.text(256 << 20, seed=2), lambda: blt_amd.BpeStrategy(m), m, \
            "f2: 256 MiB synthetic text, 4 merges two of which are valued their own first byte (generic byte pass)"
    if name == "cyclic_dense":
        # a cyclic map whose byte pass leaves a mergeable pair at every word start: (' ', c) -> ' '
        # eats one letter after each space per pass; the key (300, 301) (never made) keeps it off the
        # byte-pair-key path, so its sparse passes are tried right behind the byte pass and not taken
        # (the detect gate)
        m = {(32, c): 32 for c in range(97, 123)}
        m[(300, 301)] = 302
        return synth.text(256 << 20, seed=2), lambda: blt_amd.BpeStrategy(m), m, \
            "f2: 256 MiB synthetic text, a cyclic map ((' ', letter) -> ' ') whose passes merge densely"
    if name == "chain":
        m = synth.doubling_chain(24)
        return np.full(256 << 20, 97, np.uint8), lambda: blt_amd.BpeStrategy(m), m, \
            "f2: 256 MiB of 'a', a 24-level doubling chain: 16 MiB chunks become one token each after 24 passes"
    # wrap: the 65 537-line merges file through the loader
    import tempfile
    fd, path = tempfile.mkstemp(suffix=".txt")
    with os.fdopen(fd, "w") as f:
        f.write(synth.wrap_merges_lines())
    m = O_load(path)
    strat = blt_amd.BpeStrategy.from_file(path)
    os.unlink(path)
    return synth.text(256 << 20, seed=2), lambda: strat, m, \
        "f2: 256 MiB synthetic text, the 65 537-line merges file whose u16 ids wrap (65 536-entry map, L2 buckets)"


def O_load(path):
    from oracle import oracle as O
    return O.load_bpe_merges_from_path(path)


def general_map_rate(blt_amd, synth, O, threads, name="multi", reps=10):
    """A general map, device-resident.  `ms`: the whole asynchronous encode_device call (every
    pass enqueued, HIP events around it); `sync_ms`: the call that returns the token count (host
    wall clock), where eligible maps run passes 1 and 2 fused (`sync_path`); the output checked is
    the synchronous call's."""
    import torch
    host, make, merges, desc = general_workload(synth, name)
    n = host.size
    s = make()
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
    # the same call asking for the token count (the host waits for it): eligible maps fuse passes 1
    # and 2 into one kernel there (blt_debug_last_fused: 1 fused, 2 fell back, 0 two kernels)
    tw = []
    for _ in range(reps):
        t0 = time.perf_counter()
        s.encode_device(d_in.data_ptr(), n, CHUNK, d_out.data_ptr(), ws.data_ptr(), wsb, sp, sync=True)
        tw.append(time.perf_counter() - t0)
    sync_path = {0: "two kernels", 1: "fused passes 1+2", 2: "fused, fell back"}[int(blt_amd._lib.lib().blt_debug_last_fused())]
    got = d_out[:2 * tok].cpu().numpy()
    exp = O.COracle(merges).run(host, CHUNK, threads=threads)
    algo = n + 2 * tok
    s.close()
    return {"workload": desc, "bytes": n, "ms": round(ms, 4), "u16_passes": passes,
            "input_GBps": round(n / ms / 1e6, 1), "achieved_GBps": round(algo / ms / 1e6, 1),
            "frac": round(algo / ms / 1e6 / HBM_PEAK_GBS, 4), "tokens_per_byte": round(tok / n, 4),
            "sync_ms": round(1000 * float(np.median(tw)), 4), "sync_path": sync_path,
            "bit_exact_vs_oracle": bool(exp.size == got.size and np.array_equal(exp, got))}


def cli_phases(stderr, wall):
    """Seconds of one CLI run's phases from its BLT_CLI_TIMING lines: HIP runtime up, device tables and
    staging buffers ready, tokens written (from the run's start), and wall - tokens written (the
    process start before the run, the unmaps and the exit)."""
    import re
    st = {}
    for line in stderr.splitlines():
        m = re.match(r"blt timing: (.*?) (?:at )?\+?(-?[0-9.]+) s", line)
        if m:
            st[m.group(1)] = float(m.group(2))
    up = st.get("prewarm step: device count (runtime up)")
    ready = st.get("device ready and output preallocated")
    done = st.get("chunks written")
    out = {"runtime_up_s": up, "device_ready_s": ready, "tokens_written_s": done}
    if ready is not None and done is not None:
        out["tokenise_s"] = round(done - ready, 4)
        out["outside_run_s"] = round(wall - done, 4)
    return out


def cli_end_to_end(synth, host, merges, exp):
    """The `blt` binary on cfg3's bytes as a tmpfs file to a tmpfs output (--type text), best of 3
    after one warm run; output bytes checked against the oracle's stream."""
    import subprocess
    import tempfile
    base = "/dev/shm" if os.path.isdir("/dev/shm") else tempfile.gettempdir()
    d = tempfile.mkdtemp(prefix="blt_bench_cli_", dir=base)
    fin, fout, fm = os.path.join(d, "in.txt"), os.path.join(d, "out.bin"), os.path.join(d, "merges.txt")
    try:
        host.tofile(fin)
        with open(fm, "w") as f:
            f.write("".join(f"{a} {b}\n" for (a, b), _ in sorted(merges.items(), key=lambda kv: kv[1])))
        cmd = [os.path.join(ROOT, "blt_amd", "blt"), "-i", fin, "-o", fout, "--merges", fm, "--chunksize", "16MB",
               "--type", "text", "--gpus", "1"]
        subprocess.run(cmd, check=True, timeout=120)
        # each timed run also prints its phase stamps (BLT_CLI_TIMING: a few stderr lines)
        env = dict(os.environ, BLT_CLI_TIMING="1")
        ts, phases = [], []
        for _ in range(3):
            os.remove(fout)   # a fresh output file: O_TRUNC of the last run's pages is not the tool's cost
            t0 = time.perf_counter()
            r = subprocess.run(cmd, check=True, timeout=120, env=env, stderr=subprocess.PIPE)
            ts.append(time.perf_counter() - t0)
            phases.append(cli_phases(r.stderr.decode(errors="replace"), ts[-1]))
        got = np.fromfile(fout, dtype=np.uint8)
        ok = bool(got.size == exp.size + 2 and got[0] == 0xFF and got[1] == 0x01 and np.array_equal(got[2:], exp))
        dt = min(ts)
        return {"value": round(host.size / dt / 1e9, 3), "unit": "GB/s", "seconds": round(dt, 4),
                "seconds_all": [round(t, 4) for t in ts], "phases_all": phases, "bytes": int(host.size), "tmpfs": base,
                "path": "blt -i IN -o OUT --merges M --chunksize 16MB --type text --gpus 1 (process start to exit: "
                        "merges load, mmap, H2D, kernel, D2H, write)",
                "bit_exact_vs_oracle": ok}
    finally:
        for f in (fin, fout, fm):
            if os.path.exists(f):
                os.remove(f)
        os.rmdir(d)


def kernel_source_sha():
    import hashlib
    h = hashlib.sha256()
    for f in ("bpe_kernels.hip", "bpe_kernels.h"):
        with open(os.path.join(ROOT, "blt_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def pmc_traffic(path, wl, n):
    """HBM bytes per launch from the PMC record, only if it names this workload, size, chunk size and
    the kernel source it was measured on."""
    if not os.path.exists(path):
        return None, "no record"
    with open(path) as f:
        tj = json.load(f)
    recs = [r for k, r in tj.get("workloads", {}).items() if r.get("workload", k) == wl]
    if not recs:
        return None, f"no {wl} record"
    sized = [r for r in recs if r.get("bytes_per_gpu") == n and r.get("chunk_size") == CHUNK]
    if not sized:
        return None, "record is for another size"
    tw = sized[0]
    if tw.get("kernel_source_sha256") != kernel_source_sha():
        return None, "record is for another kernel build (kernel_source_sha256 differs)"
    return tw.get("hbm_bytes_per_launch"), tw.get("source")


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

    wl = args.workload or ("cfg3" if world == 1 else "cfg4")
    if wl == "cfg2" and distributed:
        raise SystemExit("cfg2 is a one-GPU workload")
    host, merges, wl_desc, (b0, b1), stream_bytes = workload(synth, wl, rank, world, args.bytes_per_gpu,
                                                             args.total_bytes)
    strategy = blt_amd.BpeStrategy(merges)
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

    # One reset before the first launch: the byte-scan kernel's last workgroup zeroes the ticket and
    # status words again (self-reset), so every step is the one kernel.  (A general map ignores
    # the flag and zeroes its own workspace.)
    strategy.workspace_reset(ws.data_ptr(), n, CHUNK, sp)

    def step(ev0=None, ev1=None):
        if args.reset_each_step:
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
    timed_events = not args.events_outside_timed_loop   # events over the timed region (the contract)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(*(evs[i] if timed_events else (None, None)))
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    strategy.check_workspace(ws.data_ptr(), sp)
    if not timed_events:
        # experiment: the same steps again with HIP events around each launch, so the timed loop of
        # `value` carries no event records
        for i in range(args.steps):
            step(*evs[i])
        torch.cuda.synchronize()
        strategy.check_workspace(ws.data_ptr(), sp)
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    tokens = int(d_off[-1].item())

    elapsed, kern_ms_max = shard.max_over_ranks([elapsed, kern_ms], device="cuda" if backend == "nccl" else None)
    ranges = shard.gather_ranges((b0, b1), device="cuda" if backend == "nccl" else None)
    ms_per_step = 1000.0 * elapsed / args.steps
    total_bytes = sum(r1 - r0 for r0, r1 in ranges)           # bytes all ranks processed per step
    value = total_bytes / (elapsed / args.steps) / 1e9

    algo_bytes = n + 2 * tokens                               # N + 2M per launch
    achieved = algo_bytes / (kern_ms / 1000.0) / 1e9
    traffic, traffic_src = pmc_traffic(args.traffic, wl, n)

    cpu = None
    cpu_opt = None
    exact = None
    exp = None
    usable, affinity, ncpu = usable_cores()
    threads = max(1, args.cpu_threads or usable)
    extras = {}
    if distributed and not args.no_cpu_baseline:
        # N > 1: the CPU baseline is reported at N = 1 only; EVERY rank checks its own shard
        # bit-exact against the C oracle (outside the timed region, the host cores split between
        # the ranks), and the flags are ANDed over the ranks (an all_reduce MIN of 0/1)
        from oracle import oracle as O
        exp = O.COracle(merges).run(host, CHUNK, threads=max(1, threads // world))
        got = d_out[:2 * tokens].cpu().numpy()
        mine = bool(exp.size == got.size and np.array_equal(exp, got))
        del exp, got
        exact = shard.all_ranks_true(mine, device="cuda" if backend == "nccl" else None)
    elif rank == 0 and not args.no_cpu_baseline:
        from oracle import oracle as O
        orc = O.COracle(merges)
        c0 = time.perf_counter()
        exp = orc.run(host, CHUNK, threads=threads)
        cpu_s = time.perf_counter() - c0
        cpu = {"value": round(n / cpu_s / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port",
               "usable_cores": usable, "affinity_cpus": affinity, "os_cpu_count": ncpu,
               "sample": f"the same {n >> 20} MiB {wl} shard, {nchunks} chunks of 16 MiB, C restatement "
                         f"of tokenizer.rs:56-93 (hash map, multi-pass), one task per chunk on {threads} threads "
                         f"(every usable core: min(cgroup quota, affinity mask), as num_cpus)",
               "seconds": round(cpu_s, 3)}
        got = d_out[:2 * tokens].cpu().numpy()
        exact = bool(exp.size == got.size and np.array_equal(exp, got))
        del got
        # SURVEY.md §8(d)'s "optimised CPU" line beside it: dense table, one greedy pass per chunk
        c0 = time.perf_counter()
        fast = O.fast_run(merges, host, CHUNK, threads=threads)
        fast_s = time.perf_counter() - c0
        if fast is not None:
            cpu_opt = {"value": round(n / fast_s / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port-optimized",
                       "sample": f"the same {n >> 20} MiB {wl} shard: dense 64K-entry table, one greedy "
                                 f"pass per chunk (single-pass map), {threads} threads", "seconds": round(fast_s, 3),
                       "matches_port": bool(np.array_equal(fast, exp))}
        del fast
    if rank == 0 and not distributed and not args.no_extra and wl == "cfg3":
        # the other configs (kernel-only rates) and the host paths; --only-configs runs a subset, also
        # without the CPU baseline (every row still checks its output against the oracle)
        from oracle import oracle as O
        del d_in, d_out, ws
        only = tuple(x for x in args.only_configs.split(",") if x)
        extras["configs"] = extra_configs(blt_amd, synth, O, threads, only)
        if not only:
            if exp is None:
                exp = O.COracle(merges).run(host, CHUNK, threads=threads)
            extras["end_to_end"], extras["per_chunk_path"] = host_paths(blt_amd, strategy, host, exp)
            extras["cli_end_to_end"] = cli_end_to_end(synth, host, merges, exp)

    if rank == 0:
        strong = wl in STRONG_TOTAL
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "u8",
            "data": ("synthetic: seeded uniform random bytes (splitmix64), cfg3's merges" if wl == "cfg5" else
                     "synthetic: seeded English-like text (splitmix64, 1 MiB blocks), merges ranked from it"),
            "config": {"workload": wl_desc, "stream_bytes": stream_bytes, "bytes_per_gpu": n,
                       "rank_bytes": [[int(r0), int(r1)] for r0, r1 in ranges], "chunk_size": CHUNK,
                       "merges": len(merges), "parallelism": f"chunk-sharded x{world}, no collective"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "seg::scan_bytes_kernel<true, 0, false>", "kernel_ms": round(kern_ms, 4),
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
