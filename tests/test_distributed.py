"""World-size-2 gloo tests of the one-process-per-GPU path on CPU.

Each rank tokenises its contiguous chunk range (here with the CPU oracle standing in for the
GPU), rank 0 stitches; the result must equal the single-process stream for every chunk size,
and the partition must be the one the C host library uses across devices.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from blt_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, data, merges, chunk_size, q):
    import torch.distributed as dist
    from oracle import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        orc = O.COracle(merges)

        def process(part):
            return orc.run(part, chunk_size, threads=2, return_lens=True)

        local, lens, full, full_lens = shard.run_sharded(data, chunk_size, process)
        mx = shard.max_over_ranks([float(rank + 1), float(10 - rank)])
        # bench.py's config.rank_bytes: every rank's range of cfg4's 8 GiB stream
        rg = shard.gather_ranges(shard.rank_bytes(8 << 30, 16 << 20, rank, world))
        # bench.py's per-rank bit-exact flags, ANDed over the ranks: all true, and one rank false
        ok = (shard.all_ranks_true(True), shard.all_ranks_true(rank != world - 1))
        q.put((rank, local.size, None if full is None else full.tobytes(),
               None if full_lens is None else full_lens.tolist(), mx, rg, ok))
    finally:
        dist.destroy_process_group()


def _run(world, data, merges, chunk_size):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, data, merges, chunk_size, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res)


@pytest.mark.parametrize("chunk_size", [4096, 10007, 65536])
def test_two_rank_stitch_matches_single_process(chunk_size):
    from oracle import oracle as O
    rng = np.random.default_rng(chunk_size)
    data = rng.integers(0, 6, 5 * 65536 + 321, dtype=np.uint8)
    merges = {(a, b): 256 + 6 * a + b for a in range(6) for b in range(6) if (a * 7 + b) % 3}
    res = _run(2, data, merges, chunk_size)
    full, full_lens = res[0][2], res[0][3]
    exp, elens = O.COracle(merges).run(data, chunk_size, threads=4, return_lens=True)
    assert full == exp.tobytes()
    assert full_lens == elens.tolist()
    assert res[1][2] is None
    # both ranks did work, and the max over ranks is element-wise
    assert res[0][1] > 0 and res[1][1] > 0
    assert res[0][4] == [2.0, 10.0] and res[1][4] == [2.0, 10.0]
    # every rank sees every rank's byte range, in rank order
    exp_rg = [shard.rank_bytes(8 << 30, 16 << 20, r, 2) for r in range(2)]
    assert res[0][5] == exp_rg and res[1][5] == exp_rg == [(0, 4 << 30), (4 << 30, 8 << 30)]
    # a shard that fails its check fails the run on every rank
    assert res[0][6] == res[1][6] == (True, False)


def test_partition_matches_host_library():
    # blt_host.cpp: c_lo[r] = nchunks * r / g, g = min(world, nchunks)
    for nchunks in (1, 2, 3, 7, 64, 513):
        for world in (1, 2, 4, 8):
            rs = shard.chunk_ranges(nchunks, world)
            g = max(1, min(world, nchunks))
            assert [lo for lo, _ in rs[:g]] == [nchunks * r // g for r in range(g)]
            assert rs[0][0] == 0 and max(hi for _, hi in rs) == nchunks
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))


def test_rank_bytes_weak_scaling_shards():
    # bench.py: rank r of N owns bytes [r * 1 GiB, (r + 1) * 1 GiB) of an N GiB stream
    gib, cs = 1 << 30, 16 << 20
    for world in (1, 2, 4, 8):
        for r in range(world):
            assert shard.rank_bytes(world * gib, cs, r, world) == (r * gib, (r + 1) * gib)


def test_rank_bytes_strong_scaling_shards():
    # bench.py cfg4 / cfg5: one 8 GiB (4 GiB) stream split by whole 16 MiB chunks over N ranks
    cs = 16 << 20
    for total in (8 << 30, 4 << 30):
        for world in (1, 2, 4, 8):
            per = total // world
            assert [shard.rank_bytes(total, cs, r, world) for r in range(world)] == \
                [(r * per, (r + 1) * per) for r in range(world)]
    # a stream that does not split evenly: whole chunks, the remainder on the later ranks
    n = 10 * cs + 5
    rs = [shard.rank_bytes(n, cs, r, 4) for r in range(4)]
    assert rs[0] == (0, 2 * cs) and rs[-1][1] == n
    assert all(rs[i][1] == rs[i + 1][0] for i in range(3))
    assert all((b - a) % cs == 0 for a, b in rs[:-1])


def test_bench_workload_partition():
    """bench.workload's rank ranges are shard.rank_bytes of the stream (cfg4 / cfg5 strong, cfg3
    weak), checked on small streams so no GPU or large buffer is needed."""
    import bench
    from blt_amd import synth
    for world in (2, 4):
        for r in range(world):
            _, _, desc, rg, stream = bench.workload(synth, "cfg4", r, world, total=64 << 20)
            assert rg == shard.rank_bytes(64 << 20, 16 << 20, r, world) and stream == 64 << 20
            assert desc.startswith("cfg4")
            host, _, _, rg5, _ = bench.workload(synth, "cfg5", r, world, total=32 << 20)
            assert rg5 == shard.rank_bytes(32 << 20, 16 << 20, r, world) and host.size == rg5[1] - rg5[0]
            assert np.array_equal(host, synth.random_bytes(32 << 20, seed=5)[rg5[0]:rg5[1]])
            h3, _, _, rg3, _ = bench.workload(synth, "cfg3", r, world, per_gpu=16 << 20)
            assert rg3 == (r * (16 << 20), (r + 1) * (16 << 20))
            assert np.array_equal(h3, synth.text(world * (16 << 20), seed=3)[rg3[0]:rg3[1]])
