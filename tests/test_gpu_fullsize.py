"""GPU parity at BASELINE.json's full sizes (one MI355X), through the C ABI's device entry.

- cfg5: 4 GiB of random bytes (seed 5) under cfg3's 50k merges, 16 MiB chunks, content type
  audio (0xFF02, lib.rs:93-104): the stitched stream bit-exact against the C oracle, and the
  per-chunk token counts checked against the size-independent bounds (n/2 <= M <= n per chunk,
  offsets monotone, last offset = total).
- f2: 3 GiB of text through a chained general map (u16 passes past 2^31 token bytes).
- cfg2: BASELINE's exact workload (100 MiB of seed-2 text, the 256 merges ranked from it, 16 MiB
  chunks = 7 chunks, the last one partial), stream and per-chunk offsets bit-exact.
- cfg4: 8 GiB of text cut into the 8 contiguous chunk ranges of an 8-GPU run (blt_amd.shard,
  the partition bench.py and blt_bpe_process_chunks use); every shard runs as its own launch
  and the rank-order stitch equals the one-shot oracle stream: sharding is exact.
"""
import numpy as np
import pytest

import blt_amd
from blt_amd import shard, synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu

CHUNK = 16 << 20


def _merges50k():
    return synth.merges_dict(synth.text_merges_50k(synth.text(64 << 20, seed=3), seed=3))


def _device_encode(strategy, host, cs):
    import torch
    n = host.size
    d_in = torch.from_numpy(host).cuda()
    d_out = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
    nch = (n + cs - 1) // cs
    d_off = torch.zeros(nch + 1, dtype=torch.int64, device="cuda")
    wsb = strategy.workspace_size(n, cs)
    ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    tok = strategy.encode_device(d_in.data_ptr(), n, cs, d_out.data_ptr(), ws.data_ptr(), wsb,
                                 torch.cuda.current_stream().cuda_stream, d_chunk_off=d_off.data_ptr())
    out = d_out[:2 * tok].cpu().numpy()
    off = d_off.cpu().numpy()
    del d_in, d_out, ws
    torch.cuda.empty_cache()
    return out, off


def test_cfg5_random_bytes_4gib():
    n = 4 << 30
    data = synth.random_bytes(n, seed=5)
    m = _merges50k()
    got, off = _device_encode(blt_amd.BpeStrategy(m), data, CHUNK)
    exp = O.COracle(m).run(data, CHUNK, content_type="audio", threads=16)
    assert exp[:2].tobytes() == b"\xff\x02"
    assert np.array_equal(got, exp[2:])
    lens = np.diff(off)
    sizes = np.diff(np.minimum(np.arange(off.size, dtype=np.int64) * CHUNK, n))
    assert off[0] == 0 and off[-1] == got.size // 2
    assert np.all(lens * 2 >= sizes) and np.all(lens <= sizes)


def test_cfg2_text_100mib_256_merges():
    """cfg2 exactly as bench.py builds it (bench.workload): 100 MiB of seed-2 text, the top-256
    adjacent pairs of that text as merges, --chunksize 16MB (6 whole chunks and a 4 MiB tail)."""
    n = 100 << 20
    data = synth.text(n, seed=2)
    m = synth.merges_dict(synth.top_pair_merges(data, 256))
    assert len(m) == 256
    got, off = _device_encode(blt_amd.BpeStrategy(m), data, CHUNK)
    exp, elens = O.COracle(m).run(data, CHUNK, threads=16, return_lens=True)
    assert elens.size == 7
    assert np.array_equal(got, exp)
    assert np.array_equal(np.diff(off) * 2, elens)


def test_cfg4_eight_shards_8gib():
    n = 8 << 30
    world = 8
    text = synth.text(n, seed=3)
    m = _merges50k()
    s = blt_amd.BpeStrategy(m)
    parts = []
    for r in range(world):
        b0, b1 = shard.rank_bytes(n, CHUNK, r, world)
        out, _ = _device_encode(s, text[b0:b1], CHUNK)
        parts.append(out)
    got = shard.stitch(parts)
    del parts
    exp = O.COracle(m).run(text, CHUNK, threads=16)
    assert np.array_equal(got, exp)


def test_general_map_3gib():
    """f2 at scale: 3 GiB of text through the chained, byte-valued map (one byte pass, then u16
    passes in place over ~2.9 G tokens, past 2^31 token bytes), 16 MiB chunks: stream and chunk
    offsets bit-exact against the oracle, and the chain stops after one u16 pass."""
    n = 3 << 30
    text = synth.text(n, seed=7)
    m = {(101, 32): 256, (256, 116): 257, (116, 104): 65, (65, 101): 258, (32, 116): 259, (259, 104): 260}
    got, off = _device_encode(blt_amd.BpeStrategy(m), text, CHUNK)
    assert blt_amd._lib.lib().blt_debug_last_u16_passes() == 1
    exp, elens = O.COracle(m).run(text, CHUNK, threads=16, return_lens=True)
    assert np.array_equal(got, exp)
    assert np.array_equal(np.diff(off) * 2, elens)
