"""Multi-GPU sharding of the chunked pipeline.

Chunks are independent (pipeline.rs:73-81) and chunk boundaries depend only on the chunk size,
so a stream shards into contiguous chunk ranges, one per GPU, with no collective on the data
path; the ordered stitch (pipeline.rs:153-192) is a concatenation in rank order.  The partition
is the one blt_bpe_process_chunks uses across the devices of one process (blt_host.cpp:
c_lo[r] = nchunks * r / g), so the in-process and one-process-per-GPU paths agree.

torch.distributed is used only for bookkeeping: the max over ranks of a timing and, when a
caller asks for the stitched stream on one rank, a gather of the shards (gloo on CPU, RCCL on
GPUs).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np


def num_chunks(n: int, chunk_size: int) -> int:
    if chunk_size <= 0:
        raise ValueError("chunk_size must be > 0")
    return (n + chunk_size - 1) // chunk_size


def chunk_ranges(nchunks: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous chunk ranges [lo, hi) for world ranks (blt_host.cpp c_lo[r] = nchunks*r/g)."""
    g = max(1, min(world, nchunks)) if nchunks else 1
    return [(nchunks * r // g, nchunks * (r + 1) // g) if r < g else (nchunks, nchunks) for r in range(world)]


def rank_bytes(n: int, chunk_size: int, rank: int, world: int) -> Tuple[int, int]:
    """Byte range [b0, b1) of rank's shard of an n-byte stream."""
    lo, hi = chunk_ranges(num_chunks(n, chunk_size), world)[rank]
    return min(lo * chunk_size, n), min(hi * chunk_size, n)


def stitch(parts: Sequence[np.ndarray]) -> np.ndarray:
    """Ordered stitch: shard outputs in rank (= chunk) order."""
    parts = [np.asarray(p, dtype=np.uint8) for p in parts]
    return np.concatenate(parts) if parts else np.zeros(0, np.uint8)


def max_over_ranks(values: Sequence[float], device=None) -> List[float]:
    """Element-wise max over ranks (identity without an initialised process group)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.cpu()]


def all_ranks_true(flag: bool, device=None) -> bool:
    """AND of a per-rank flag over every rank (the flag itself without a process group)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if flag else 0], dtype=torch.int64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t.item()))


def gather_ranges(rng: Tuple[int, int], device=None) -> List[Tuple[int, int]]:
    """Every rank's (b0, b1), in rank order (this rank's alone without a process group)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return [tuple(int(x) for x in rng)]
    t = torch.tensor(list(rng), dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [(int(a), int(b)) for a, b in (o.cpu().tolist() for o in out)]


def run_sharded(data: np.ndarray, chunk_size: int, process: Callable[[np.ndarray], Tuple[np.ndarray, np.ndarray]],
                gather: bool = True) -> Tuple[np.ndarray, np.ndarray, Optional[np.ndarray], Optional[np.ndarray]]:
    """Tokenises this rank's shard with process(shard) -> (tokens_be_bytes, chunk_lens) and, with
    gather, returns the stitched stream and chunk lengths on rank 0 (None elsewhere).

    process is the GPU path in production (BpeStrategy.process_chunks on the rank's device);
    any function with the same contract works (the CPU tests pass the oracle).
    """
    import torch.distributed as dist
    distributed = dist.is_available() and dist.is_initialized()
    rank = dist.get_rank() if distributed else 0
    world = dist.get_world_size() if distributed else 1
    b0, b1 = rank_bytes(data.size, chunk_size, rank, world)
    out, lens = process(data[b0:b1])
    out = np.asarray(out, dtype=np.uint8)
    lens = np.asarray(lens, dtype=np.int64)
    if not gather:
        return out, lens, None, None
    if world == 1:
        return out, lens, out, lens
    objs = [None] * world if rank == 0 else None
    dist.gather_object((out, lens), objs, dst=0)
    if rank != 0:
        return out, lens, None, None
    return out, lens, stitch([o for o, _ in objs]), np.concatenate([l for _, l in objs])
