"""Round 6: no kernel reads or writes outside its buffers, and a broken count is a flagged error.

* Guard pages (VERDICT r5 weak #1 / "next" #1).  Round 5's intermittent "illegal memory access"
  (ASan driver, trial 3: a general map of chain depth 2, 70001 bytes, chunk size 65537) came from
  the fused passes 1 + 2 (``seg::load_fused``): a wave range past the input's end still loaded the
  64-byte halo before it, up to ~32 KiB past the input.  It faulted only when the input's device
  allocation was exactly ``up16(n)`` bytes long (a pooled staging context regrown for that n) and
  the pages after it were unmapped.  Here the input and the output end at the end of a mapped HIP
  virtual-memory granule whose successor is reserved and left unmapped, so any access past them
  faults at once, on every run.  Each strategy path runs
  on such buffers: the byte pass (a merges file), the fused passes of that trial's map, the u16
  scan passes and the finish kernel of a chained map, the sparse passes of a cyclic map.
  Bit-exact against the oracle.  (The basic strategy's loads are whole 8-byte blocks below n and
  single bytes below n: not tested here.  Freshly remapped granules of a few KiB were seen to hand a
  kernel stale bytes after a host-to-device copy, a property of the runtime's VMM mappings, not of
  the kernels: the strategy cases use one input mapping per case.)
* Injected counts (``blt_debug_set_inject``).  The finish kernel, the u16 scan and the sparse
  compaction each break one of their counts on purpose; their invariant checks must turn it into
  BLT_E_IO (the handle's sticky error) with nothing written outside the count's range, and the
  process's HIP context must survive: after ``clear_error`` the same call is bit-exact.
"""
import ctypes

import numpy as np
import pytest

import blt_amd
from blt_amd import _lib, synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu


# ---- HIP virtual memory: buffers that end where a mapped granule ends ------------------------
class _Loc(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("id", ctypes.c_int)]


class _Flags(ctypes.Structure):
    _fields_ = [("compressionType", ctypes.c_ubyte), ("gpuDirectRDMACapable", ctypes.c_ubyte),
                ("usage", ctypes.c_ushort)]


class _Prop(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("requestedHandleType", ctypes.c_int), ("location", _Loc),
                ("win32HandleMetaData", ctypes.c_void_p), ("allocFlags", _Flags)]


class _Access(ctypes.Structure):
    _fields_ = [("location", _Loc), ("flags", ctypes.c_int)]


def _hip():
    """The HIP runtime the library and torch use (torch's bundled copy when there is one, as
    blt_amd._lib loads it): another libamdhip64.so would be a second runtime in the process, whose
    memsets and synchronisations the library's streams never see."""
    import os
    import torch
    path = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    _lib.lib()
    h = ctypes.CDLL(path if os.path.exists(path) else "libamdhip64.so")
    for name in ("hipMemGetAllocationGranularity", "hipMemAddressReserve", "hipMemCreate", "hipMemMap",
                 "hipMemSetAccess", "hipMemUnmap", "hipMemRelease", "hipMemAddressFree", "hipMemcpy",
                 "hipDeviceSynchronize", "hipGetDevice", "hipMemset"):
        getattr(h, name).restype = ctypes.c_int
    return h


class GuardedBuffer:
    """`size` device bytes whose last byte is the last mapped byte of a HIP VMM granule: the next
    granule is reserved and never mapped, so a read or write past the buffer faults."""

    def __init__(self, hip, size):
        self.hip = hip
        dev = ctypes.c_int(0)
        assert hip.hipGetDevice(ctypes.byref(dev)) == 0
        self.prop = _Prop(type=1, requestedHandleType=0, location=_Loc(type=1, id=dev.value))
        gran = ctypes.c_size_t(0)
        assert hip.hipMemGetAllocationGranularity(ctypes.byref(gran), ctypes.byref(self.prop), 0) == 0
        g = gran.value
        self.size = size
        self.mapped = max(g, (size + g - 1) // g * g)
        self.reserved = self.mapped + g
        self.va = ctypes.c_void_p(0)
        assert hip.hipMemAddressReserve(ctypes.byref(self.va), ctypes.c_size_t(self.reserved),
                                        ctypes.c_size_t(0), None, ctypes.c_ulonglong(0)) == 0
        self.handle = ctypes.c_void_p(0)
        assert hip.hipMemCreate(ctypes.byref(self.handle), ctypes.c_size_t(self.mapped), ctypes.byref(self.prop),
                                ctypes.c_ulonglong(0)) == 0
        assert hip.hipMemMap(self.va, ctypes.c_size_t(self.mapped), ctypes.c_size_t(0), self.handle,
                             ctypes.c_ulonglong(0)) == 0
        acc = _Access(location=_Loc(type=1, id=dev.value), flags=3)
        assert hip.hipMemSetAccess(self.va, ctypes.c_size_t(self.mapped), ctypes.byref(acc), ctypes.c_size_t(1)) == 0
        # 16-byte aligned start; the buffer's end is at most 15 bytes short of the granule's end
        self.ptr = self.va.value + self.mapped - ((size + 15) // 16 * 16)
        assert self.ptr % 16 == 0

    def upload(self, data: np.ndarray):
        a = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
        assert a.size <= self.size
        assert self.hip.hipMemcpy(ctypes.c_void_p(self.ptr), a.ctypes.data_as(ctypes.c_void_p),
                                  ctypes.c_size_t(a.size), 1) == 0
        # (a copy from pageable memory may return before its DMA has landed)
        assert self.hip.hipDeviceSynchronize() == 0

    def fill(self, byte):
        assert self.hip.hipMemset(ctypes.c_void_p(self.ptr), ctypes.c_int(byte), ctypes.c_size_t(self.size)) == 0
        assert self.hip.hipDeviceSynchronize() == 0   # (hipMemset may return before the memory is set)

    def download(self, n, dtype=np.uint8):
        out = np.empty(n * np.dtype(dtype).itemsize, np.uint8)
        assert self.hip.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(self.ptr),
                                  ctypes.c_size_t(out.size), 2) == 0
        return out.view(dtype)

    def free(self):
        self.hip.hipDeviceSynchronize()
        self.hip.hipMemUnmap(self.va, ctypes.c_size_t(self.mapped))
        self.hip.hipMemRelease(self.handle)
        self.hip.hipMemAddressFree(self.va, ctypes.c_size_t(self.reserved))


def _trial3_map():
    """The sanitizer driver's trial-3 map kind: keys (a < 13, 256 + k), values >= 256, chain depth 2
    (an acyclic general map: the fused passes 1 + 2 and chain_final_kernel only, no finish kernel)."""
    rng = np.random.default_rng(3)
    m = {}
    for _ in range(40):
        m[(int(rng.integers(0, 13)), 256 + int(rng.integers(0, 8)))] = 256 + int(rng.integers(0, 64))
    return m


def _cases():
    text = synth.text(300_001, seed=5)
    rng = np.random.default_rng(11)
    small = rng.integers(0, 13, 70_001, dtype=np.uint8)
    runs = np.full(200_003, 97, np.uint8)
    runs[rng.choice(runs.size, 2000, replace=False)] = 98
    return {
        "merges_file": (synth.merges_dict(synth.top_pair_merges(text, 256)), text, (65537, 4096, 1 << 20)),
        "trial3_fused": (_trial3_map(), small, (65537, 4096, 70001)),
        "trial3_text_bytes": (_trial3_map(), text, (65537, 4099)),
        "chained_text": (synth.CHAINED_TEXT_MAP, text, (65537, 1 << 20, 4099)),
        "doubling_chain_finish": (synth.doubling_chain(8), runs, (32768, 1000)),
        "self_valued_sparse": (synth.SELF_VALUED_MAP, text, (65537, 1 << 18)),
    }


@pytest.fixture(scope="module")
def hip():
    import torch
    assert torch.cuda.is_available()
    torch.cuda.init()
    return _hip()


@pytest.mark.parametrize("case", ["merges_file", "trial3_fused", "trial3_text_bytes", "chained_text",
                                  "doubling_chain_finish", "self_valued_sparse"])
def test_no_access_past_buffers(hip, case):
    import torch
    m, data, chunk_sizes = _cases()[case]
    s = blt_amd.BpeStrategy(m)
    n = data.size
    d_in = GuardedBuffer(hip, n)
    d_in.upload(data)
    try:
        for cs in chunk_sizes:
            exp, elens = O.COracle(m).run(data, cs, threads=8, return_lens=True)
            nch = (n + cs - 1) // cs
            wsb = s.workspace_size(n, cs)
            # the input (read by every kernel) and the output (written by every kernel) end at a
            # granule's end; the workspace and the chunk offsets, which the library also memsets and
            # copies with the HIP runtime's own calls, are ordinary allocations of their exact size
            d_out = GuardedBuffer(hip, 2 * n)
            try:
                for sync in (True, False):
                    d_out.fill(0)
                    ws = torch.full((wsb,), 0x5A, dtype=torch.uint8, device="cuda")
                    d_off = torch.full((nch + 1,), -1, dtype=torch.int64, device="cuda")
                    torch.cuda.synchronize()
                    stream = torch.cuda.current_stream().cuda_stream
                    tok = s.encode_device(d_in.ptr, n, cs, d_out.ptr, ws.data_ptr(), wsb, stream, d_off.data_ptr(),
                                          sync=sync)
                    torch.cuda.synchronize()
                    if sync:
                        assert tok * 2 == exp.size, (case, cs)
                    offs = d_off.cpu().numpy()
                    assert int(offs[-1]) * 2 == exp.size, (case, cs, sync)
                    assert np.array_equal(d_out.download(exp.size), exp), (case, cs, sync)
                    assert np.array_equal(np.diff(offs) * 2, elens), (case, cs, sync)
                    s.check_workspace(ws.data_ptr(), stream)
            finally:
                d_out.free()
    finally:
        d_in.free()


# ---- injected counts ---------------------------------------------------------------------------
_INJECT = {"finish": 1, "fused": 2, "scan_tokens": 2, "sparse_move": 4}


def _inject_case(kind):
    """(map, data, chunk size, debug switches, the error flags the check raises)"""
    text = synth.text((2 << 20) + 91, seed=29)
    if kind == "finish":        # a depth-8 chain, 4099-byte chunks: the finish kernel from u16 pass 2 on
        runs = np.full((2 << 20) + 91, 97, np.uint8)
        runs[np.random.default_rng(7).choice(runs.size, 20000, replace=False)] = 98
        return synth.doubling_chain(8), runs, 4099, {"finish": 1, "fused": 1}, "flags 0x40"
    if kind == "fused":         # chain depth 2: the fused passes 1 + 2 are the whole chain
        return synth.CHAINED_TEXT_MAP, text, 1 << 20, {"finish": 1, "fused": 1}, "flags 0x4"
    if kind == "scan_tokens":   # no fused kernel, no finish kernel: the byte pass, then a u16 scan pass
        return synth.CHAINED_TEXT_MAP, text, 1 << 20, {"finish": 0, "fused": 0}, "flags 0x4"
    return synth.SELF_VALUED_MAP, text, 1 << 20, {"finish": 1, "fused": 1}, "flags 0x4"   # the compaction


@pytest.mark.parametrize("kind", ["finish", "fused", "scan_tokens", "sparse_move"])
@pytest.mark.parametrize("api", ["host", "device"])
def test_injected_count_is_flagged(kind, api):
    """A count broken inside the kernel (blt_debug_set_inject) is caught by the kernel's invariant
    check: the call fails with BLT_E_IO and the error names the check, the output past the correct
    token count is untouched (device API), and after clear_error the same call is bit-exact in the
    same process (no device fault)."""
    import torch
    L = _lib.lib()
    m, data, cs, opts, flags = _inject_case(kind)
    s = blt_amd.BpeStrategy(m)
    exp = O.COracle(m).run(data, cs, threads=8)
    prev_f = L.blt_debug_set_finish(opts["finish"])
    prev_sp = L.blt_debug_set_sparse(1)
    L.blt_debug_set_fused(opts["fused"])
    n = data.size
    try:
        L.blt_debug_set_inject(_INJECT[kind])
        try:
            if api == "host":
                with pytest.raises(blt_amd.BltError) as ei:
                    s.process_chunks(data, cs)
            else:
                d_in = torch.from_numpy(data).cuda()
                d_out = torch.full((2 * n + 4096,), 0xA5, dtype=torch.uint8, device="cuda")
                wsb = s.workspace_size(n, cs)
                ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
                stream = torch.cuda.current_stream().cuda_stream
                with pytest.raises(blt_amd.BltError) as ei:
                    s.encode_device(d_in.data_ptr(), n, cs, d_out.data_ptr(), ws.data_ptr(), wsb, stream, sync=True)
                torch.cuda.synchronize()
                # nothing past the input's worth of output (2n bytes) was written
                assert bool((d_out[2 * n:] == 0xA5).all().item())
        finally:
            L.blt_debug_set_inject(0)
        assert ei.value.code == _lib.BLT_E_IO, ei.value
        msg = str(ei.value)
        assert flags + " " in msg or flags + ":" in msg, msg   # the check that caught it
        assert s.clear_error() is True                         # the handle's sticky error was set
        got = s.process_chunks(data, cs)
        assert np.array_equal(got, exp), kind
        assert not s.clear_error()
    finally:
        L.blt_debug_set_inject(0)
        L.blt_debug_set_finish(prev_f)
        L.blt_debug_set_sparse(prev_sp)
        L.blt_debug_set_fused(1)
