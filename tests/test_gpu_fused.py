"""Passes 1 and 2 of a general map in one kernel (seg::scan_tokens_kernel<kHash, true>), against the
oracle and against the two-kernel chain: wave-range carries from the 64-byte halo, chunk starts at
every offset the front end distinguishes, the next range's first token, buffer ends, and the
fallback when a halo holds no restart (tokenizer.rs:63-86)."""
import contextlib
import random

import numpy as np
import pytest

import blt_amd
from blt_amd import _lib, synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fused_for_cyclic_maps():
    """The fused kernel's tests keep it for cyclic maps too: the sparse passes off (by default a
    cyclic map takes the byte pass and then the sparse passes, no fused kernel)."""
    prev = _lib.lib().blt_debug_set_sparse(0)
    yield
    _lib.lib().blt_debug_set_sparse(prev)

CHAINED_TEXT_MAP = synth.CHAINED_TEXT_MAP


def _last_fused():
    return _lib.lib().blt_debug_last_fused()


@contextlib.contextmanager
def two_kernels():
    _lib.lib().blt_debug_set_fused(0)
    try:
        yield
    finally:
        _lib.lib().blt_debug_set_fused(1)


def _check(m, data, cs, want_fused=1):
    s = blt_amd.BpeStrategy(m)
    got, lens = s.process_chunks(data, cs, return_chunk_lens=True)
    used = _last_fused()
    exp, elens = O.COracle(m).run(data, cs, threads=8, return_lens=True)
    assert np.array_equal(got, exp)
    assert np.array_equal(lens, elens)
    if want_fused is not None:
        assert used == want_fused, used
    return got


@pytest.mark.parametrize("cs", [4096, 4097, 5119, 65536, 65536 + 1023, 65536 + 1024, 65536 + 1025,
                                65536 + 1088, (1 << 20) + 63, 1 << 20])
def test_fused_chained_text_chunk_offsets(cs):
    """The chained text map (byte and token keys) over odd chunk sizes: chunk starts at offsets 0, 1,
    1023, 1024 (the next range's first byte), 1025 and inside the halo of the following range."""
    text = synth.text((3 << 20) + 777, seed=41)
    _check(CHAINED_TEXT_MAP, text, cs)


def test_fused_chunk_start_at_every_range_offset():
    """Chunk size 1024 * 7 + 1: over the buffer, the chunk starts walk through every byte offset of a
    wave range once."""
    text = synth.text(9 << 20, seed=42)
    _check(CHAINED_TEXT_MAP, text, 1024 * 7 + 1)


@pytest.mark.parametrize("n", [1, 2, 1023, 1024, 1025, 1026, 4095, 4096, 4097, 16383, 16384, 16385,
                               32767, 32768, 32769, 3 * 32768 + 5])
def test_fused_buffer_ends(n):
    text = synth.text(n, seed=n)
    got = _check(CHAINED_TEXT_MAP, text, 4096, want_fused=None)
    assert got.size == O.COracle(CHAINED_TEXT_MAP).run(text, 4096, threads=1).size


def test_fused_merges_across_range_boundaries():
    """Pairs straddling every wave-range boundary: a pass-1 merge of bytes 1023 and 1024 (the next
    range's first byte consumed), and a pass-2 merge of the range's last token with the next
    range's first token."""
    data = bytearray(synth.text(2 << 20, seed=43).tobytes())
    for b in range(1024, len(data) - 4, 1024):
        if (b // 1024) % 2:
            data[b - 1], data[b] = 101, 32            # "e" | " ": pass-1 merge across the boundary
        else:
            data[b - 2:b + 2] = b"e th"               # "e " then "t": 256 | 116 -> 257 across it
    data = np.frombuffer(bytes(data), np.uint8)
    for cs in (1 << 20, 4096 + 1024):
        _check(CHAINED_TEXT_MAP, data, cs)


def test_fused_matches_two_kernel_chain():
    """The same calls with the fused kernel and with the two-kernel chain give the same bytes."""
    text = synth.text((5 << 20) + 3, seed=44)
    s = blt_amd.BpeStrategy(CHAINED_TEXT_MAP)
    a = s.process_chunks(text, 1 << 20)
    assert _last_fused() == 1
    with two_kernels():
        b = s.process_chunks(text, 1 << 20)
        assert _last_fused() == 0
    assert np.array_equal(a, b)


@pytest.mark.parametrize("cs", [1 << 18, 4096 * 3 + 7])
def test_fused_halo_fallback(cs):
    """Runs of merging pairs longer than the halo ("abab...", with both (a, b) and (b, a) keys):
    the fused kernel cannot resolve those wave ranges, flags it, and the host runs the two-kernel
    chain (a cyclic map: the host-checked path; with a bounded chain: the check after the fused
    kernel)."""
    data = np.frombuffer(b"ab" * ((1 << 19) + 3), np.uint8).copy()
    data[::5003] = 99
    for m in ({(97, 98): 256, (98, 97): 257, (256, 256): 258, (258, 99): 259},
              {(97, 98): 256, (98, 97): 98, (256, 98): 260}):
        _check(m, data, cs, want_fused=2)


def test_fused_not_tried_for_byte_self_pairs():
    """A map with a byte-pair key (a, a) (runs of one byte merge pair after pair) keeps the
    two-kernel chain."""
    m = {(97, 97): 256, (256, 98): 257, (98, 98): 258}
    data = np.full((1 << 20) + 5, 97, np.uint8)
    data[::4099] = 98
    _check(m, data, 1 << 18, want_fused=0)


@pytest.mark.parametrize("seed", range(16))
def test_fused_random_general_maps(seed):
    """Random general maps (byte-valued, new and near-top ids, chains) over skewed text-like bytes
    with enough distinct pairs that the halo usually restarts: fused or fallen back, always exact."""
    rng = random.Random(2000 + seed)
    alph = rng.choice([6, 12, 26])
    letters = [97 + i for i in range(alph)] + [32]
    toks = list(letters)
    m = {}
    nxt = rng.choice([256, 300, 65500])
    for _ in range(rng.randrange(4, 80)):
        a, b = rng.choice(toks), rng.choice(toks)
        if (a, b) in m:
            continue
        v = rng.choice(letters) if rng.random() < 0.1 else (nxt & 0xFFFF)
        if v == (nxt & 0xFFFF):
            nxt += 1
        m[(a, b)] = v
        if v not in toks and rng.random() < 0.7:
            toks.append(v)
    if all(a < 256 and b < 256 for a, b in m):
        m[(toks[-1] if toks[-1] >= 256 else 256, 97)] = 60000   # a token key: not a byte-pair-only map
    w = np.array([rng.random() ** 2 + 0.02 for _ in letters])
    n = rng.choice([(1 << 19) + 3, (2 << 20) + 17])
    data = np.random.default_rng(seed).choice(np.array(letters, np.uint8), n, p=w / w.sum())
    cs = rng.choice([4096, 4097, 12289, 65536, (1 << 20) + 1])
    _check(m, data, cs, want_fused=None)
    assert _last_fused() in ((0,) if any(a == b < 256 for a, b in m) else (1, 2))


def test_fused_device_api_sync_and_async():
    """encode_device: a synchronous call (token count asked for) fuses; an asynchronous one keeps the
    two-kernel chain; both give the oracle's tokens and chunk offsets."""
    import torch
    data = synth.text((4 << 20) + 9, seed=45)
    s = blt_amd.BpeStrategy(CHAINED_TEXT_MAP)
    cs = 1 << 20
    n = data.size
    nchunks = (n + cs - 1) // cs
    d_in = torch.from_numpy(data).cuda()
    d_out = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
    d_off = torch.zeros(nchunks + 1, dtype=torch.int64, device="cuda")
    ws_b = s.workspace_size(n, cs)
    ws = torch.empty(ws_b, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    exp, elens = O.COracle(CHAINED_TEXT_MAP).run(data, cs, threads=8, return_lens=True)
    tok = s.encode_device(d_in.data_ptr(), n, cs, d_out.data_ptr(), ws.data_ptr(), ws_b, stream,
                          d_off.data_ptr(), sync=True)
    assert _last_fused() == 1
    assert 2 * tok == exp.size and np.array_equal(d_out[:2 * tok].cpu().numpy(), exp)
    assert np.array_equal(np.diff(d_off.cpu().numpy()) * 2, elens)
    d_out.zero_()
    s.encode_device(d_in.data_ptr(), n, cs, d_out.data_ptr(), ws.data_ptr(), ws_b, stream, d_off.data_ptr(),
                    sync=False)
    torch.cuda.synchronize()
    assert np.array_equal(d_out[:exp.size].cpu().numpy(), exp)
    assert np.array_equal(np.diff(d_off.cpu().numpy()) * 2, elens)
