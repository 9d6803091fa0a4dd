"""blt_amd — MI355X-native BPE merge scan, a drop-in for jtrefon/blt's BPE strategy path.

Python mirror of the reference's strategy surface over the C ABI in include/blt_bpe.h:

* ``TokenizationStrategy.process_chunk(chunk) -> bytes``   (blt_core/src/tokenizer.rs:21-31)
* ``BpeStrategy(merges)`` / ``BpeStrategy.new(merges)``     (tokenizer.rs:43-93)
* ``BasicTokenizationStrategy``                             (tokenizer.rs:96-124)
* ``load_bpe_merges_from_path`` / ``load_bpe_merges``       (config_loader.rs:14-46, lib.rs:216-230)
* ``parse_chunk_size_str``, ``get_effective_chunk_size``, ``determine_thread_count``
  (utils.rs:10-45, chunking.rs:26-62, utils.rs:79-97)
* ``BpeStrategy.process_chunks(data, chunk_size, n_gpus)``  — the mmap pipeline's chunk split and
  ordered stitch (pipeline.rs:56-192), sharded over GPUs.
* ``PassthroughStrategy``, ``select_strategy``, ``run_tokenizer`` — strategy choice
  (lib.rs:271-282), content-type token (lib.rs:284-293) and the chunked pipeline over a buffer.
* ``ByteTokenizer(merges, content_type, threads, chunk_size, memory_cap).tokenize_file(in, out)``,
  ``load_bpe_merges``, ``version``, ``__version__`` — the reference's Python binding
  (blt_python/src/lib.rs:27-220, blt_python/python/blt/__init__.py); ``tokenize_file`` runs the
  file pipeline in the library (``blt_run_tokenizer``, the one the ``blt`` CLI runs).

All tokenising calls run the HIP kernels in libblt_bpe.so; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import json
import os
from typing import Dict, Optional, Tuple

from . import _lib
from ._lib import BltError

__all__ = [
    "ByteTokenizer", "__version__", "file_tokenizer",
    "BltError", "TokenizationStrategy", "BpeStrategy", "BasicTokenizationStrategy", "PassthroughStrategy",
    "ContentType", "select_strategy", "run_tokenizer",
    "load_bpe_merges_from_path", "load_bpe_merges", "parse_chunk_size_str", "get_effective_chunk_size",
    "determine_thread_count", "version",
]


def version() -> str:
    """version() (blt_python/src/lib.rs:212-215): the library's semantic version."""
    return _lib.lib().blt_version().decode().split()[-1]


class ContentType:
    """ContentType::get_token_value — blt_core/src/lib.rs:93-104."""
    Text = 0xFF01
    Audio = 0xFF02
    Bin = 0xFF03
    Video = 0xFF04
    BY_NAME = {"text": Text, "audio": Audio, "bin": Bin, "video": Video}


def _buf(data):
    """(address, length, keepalive) of a bytes-like / numpy uint8 object."""
    try:
        import numpy as np
        if isinstance(data, np.ndarray):
            a = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
            return a.ctypes.data, a.size, a
    except ImportError:  # pragma: no cover
        pass
    mv = memoryview(data).cast("B")
    if mv.readonly:
        b = ctypes.create_string_buffer(bytes(mv), max(len(mv), 1))
        return ctypes.addressof(b), len(mv), b
    b = (ctypes.c_uint8 * max(len(mv), 1)).from_buffer(mv) if len(mv) else (ctypes.c_uint8 * 1)()
    return ctypes.addressof(b), len(mv), (b, mv)


def load_bpe_merges_from_path(path: str) -> Dict[Tuple[int, int], int]:
    """config_loader.rs:14-46.  Raises BltError (kind NotFound / InvalidData / Other)."""
    L = _lib.lib()
    cap = 65536
    A = (ctypes.c_uint16 * cap)()
    B = (ctypes.c_uint16 * cap)()
    V = (ctypes.c_uint16 * cap)()
    n = ctypes.c_size_t(0)
    _lib.check(L.blt_load_bpe_merges(str(path).encode(), A, B, V, cap, ctypes.byref(n)))
    return {(A[i], B[i]): V[i] for i in range(n.value)}


def load_bpe_merges(path: str) -> Dict[Tuple[int, int], int]:
    """blt_core::load_bpe_merges (lib.rs:216-230): the file's map with (u8, u8) keys."""
    return {k: v for k, v in load_bpe_merges_from_path(path).items() if k[0] <= 255 and k[1] <= 255}


def parse_chunk_size_str(s: str) -> int:
    """utils.rs:10-45.  Raises ValueError with the reference's message."""
    out = ctypes.c_uint64(0)
    L = _lib.lib()
    if L.blt_parse_chunk_size(s.encode(), ctypes.byref(out)) != 0:
        raise ValueError(L.blt_last_error().decode())
    return out.value


def get_effective_chunk_size(cli_chunk_size: Optional[int], num_threads: int, mem_cap_percent: int = 80) -> int:
    """chunking.rs:26-62 (dynamic branch reads /proc/meminfo, like sysinfo's total_memory)."""
    return _lib.lib().blt_effective_chunk_size(int(cli_chunk_size is not None), cli_chunk_size or 0,
                                               num_threads, mem_cap_percent)


def determine_thread_count(threads: Optional[int]) -> int:
    """utils.rs:79-97."""
    return _lib.lib().blt_determine_thread_count(int(threads is not None), threads or 0)


class TokenizationStrategy:
    """trait TokenizationStrategy (tokenizer.rs:21-31): process one chunk of bytes."""

    def process_chunk(self, chunk_data) -> bytes:  # pragma: no cover - interface
        raise NotImplementedError


class BpeStrategy(TokenizationStrategy):
    """BpeStrategy (tokenizer.rs:33-94) on the GPU.

    ``merges`` is a BpeMerges map {(u16, u16): u16} (lib.rs:75).  The handle is immutable and
    safe to share between threads, like the reference's Arc<dyn TokenizationStrategy>.
    """

    def __init__(self, merges: Optional[Dict[Tuple[int, int], int]] = None, *, _handle=None):
        self._L = _lib.lib()
        self._h = ctypes.c_void_p()
        if _handle is not None:
            self._h = _handle
        else:
            items = list((merges or {}).items())
            n = len(items)
            A = (ctypes.c_uint16 * max(n, 1))(*[int(k[0]) for k, _ in items])
            B = (ctypes.c_uint16 * max(n, 1))(*[int(k[1]) for k, _ in items])
            V = (ctypes.c_uint16 * max(n, 1))(*[int(v) for _, v in items])
            _lib.check(self._L.blt_bpe_create(A, B, V, n, 0, ctypes.byref(self._h)))

    @classmethod
    def new(cls, bpe_merges: Dict[Tuple[int, int], int]) -> "BpeStrategy":
        """BpeStrategy::new(Arc<BpeMerges>) — tokenizer.rs:48."""
        return cls(bpe_merges)

    @classmethod
    def from_file(cls, merges_path: str) -> "BpeStrategy":
        """CoreConfig::load_bpe_data + select_strategy (lib.rs:184-201, :271-282)."""
        L = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(L.blt_bpe_create_from_file(str(merges_path).encode(), ctypes.byref(h)))
        return cls(_handle=h)

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            self._L.blt_bpe_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover
            pass

    @property
    def handle(self) -> int:
        return self._h.value

    def info(self) -> Tuple[int, bool]:
        n = ctypes.c_size_t(0)
        sp = ctypes.c_int(0)
        _lib.check(self._L.blt_bpe_info(self._h, ctypes.byref(n), ctypes.byref(sp)))
        return n.value, bool(sp.value)

    def process_chunk(self, chunk_data) -> bytes:
        """TokenizationStrategy::process_chunk (tokenizer.rs:56-93): BE u16 token bytes."""
        ptr, n, keep = _buf(chunk_data)
        out = ctypes.create_string_buffer(max(2 * n, 1))
        olen = ctypes.c_size_t(0)
        _lib.check(self._L.blt_bpe_process_chunk(self._h, ptr, n, out, 2 * n, ctypes.byref(olen)))
        return out.raw[:olen.value]

    def process_chunks(self, data, chunk_size: int, n_gpus: int = 1, return_chunk_lens: bool = False):
        """Chunk split + per-chunk BPE + ordered concatenation (pipeline.rs:73-81, :153-192)."""
        import numpy as np
        ptr, n, keep = _buf(data)
        out = np.empty(max(2 * n, 1), dtype=np.uint8)
        nchunks = (n + chunk_size - 1) // chunk_size if n else 0
        lens = np.zeros(max(nchunks, 1), dtype=np.uint64)
        olen = ctypes.c_size_t(0)
        _lib.check(self._L.blt_bpe_process_chunks(self._h, ptr, n, chunk_size, n_gpus, out.ctypes.data, 2 * n,
                                                  ctypes.byref(olen), lens.ctypes.data))
        res = out[:olen.value]
        if return_chunk_lens:
            return res, lens[:nchunks].astype(np.int64)
        return res

    # ---- device-resident API (pointers are integers, e.g. torch tensor .data_ptr()) ----
    def workspace_size(self, n: int, chunk_size: int) -> int:
        return self._L.blt_bpe_workspace_size(self._h, n, chunk_size)

    def encode_device(self, d_in: int, n: int, chunk_size: int, d_out: int, d_workspace: int,
                      workspace_bytes: int, stream: int = 0, d_chunk_off: int = 0, sync: bool = True):
        """blt_bpe_encode_device: returns the token count when sync, else None (async enqueue)."""
        tok = ctypes.c_uint64(0)
        _lib.check(self._L.blt_bpe_encode_device(self._h, d_in, n, chunk_size, d_out, d_chunk_off or None,
                                                 d_workspace, workspace_bytes, stream or None,
                                                 ctypes.byref(tok) if sync else None))
        return tok.value if sync else None

    def workspace_reset(self, d_workspace: int, n: int, chunk_size: int, stream: int = 0) -> None:
        _lib.check(self._L.blt_bpe_workspace_reset(self._h, d_workspace, n, chunk_size, stream or None))

    def encode_device_prezeroed(self, d_in: int, n: int, chunk_size: int, d_out: int, d_workspace: int,
                                workspace_bytes: int, stream: int = 0, d_chunk_off: int = 0) -> None:
        """Enqueues only the merge-scan kernel.  The workspace's look-back words must be zero: a
        workspace_reset for an n at least this one on the stream since the last encode, or
        single-pass encodes last (each kernel leaves its words zeroed).  A launch over more tiles
        than the workspace is known zeroed for refuses (writes nothing, error bit 32: the next
        check_workspace raises and the handle's next call fails until clear_error)."""
        _lib.check(self._L.blt_bpe_encode_device_ex(self._h, d_in, n, chunk_size, d_out, d_chunk_off or None,
                                                    d_workspace, workspace_bytes, stream or None, None, 1))

    def clear_error(self) -> bool:
        """blt_bpe_clear_error: resets the handle's sticky device error (every call fails with
        BltError(BLT_E_IO) after a kernel of the handle flagged one).  True if one was pending."""
        rc = self._L.blt_bpe_clear_error(self._h)
        if rc not in (0, _lib.BLT_E_IO):
            _lib.check(rc)
        return rc == _lib.BLT_E_IO

    def check_workspace(self, d_workspace: int, stream: int = 0) -> None:
        _lib.check(self._L.blt_bpe_check_workspace(d_workspace, stream or None))


class BasicTokenizationStrategy(TokenizationStrategy):
    """BasicTokenizationStrategy (tokenizer.rs:96-124) on the GPU: byte b -> BE [0, b]."""

    def __init__(self):
        self._L = _lib.lib()

    def process_chunk(self, chunk_data) -> bytes:
        ptr, n, keep = _buf(chunk_data)
        out = ctypes.create_string_buffer(max(2 * n, 1))
        olen = ctypes.c_size_t(0)
        _lib.check(self._L.blt_basic_process_chunk(ptr, n, out, 2 * n, ctypes.byref(olen)))
        return out.raw[:olen.value]

    def encode_device(self, d_in: int, n: int, d_out: int, stream: int = 0) -> None:
        _lib.check(self._L.blt_basic_encode_device(d_in, n, d_out, stream or None))


class PassthroughStrategy(TokenizationStrategy):
    """PassthroughStrategy (tokenizer.rs:126-145): returns the chunk unchanged (copy mode)."""

    def process_chunk(self, chunk_data) -> bytes:
        return bytes(memoryview(chunk_data).cast("B"))


def select_strategy(bpe_merges: Optional[Dict[Tuple[int, int], int]] = None, passthrough: bool = False):
    """select_strategy (lib.rs:271-282): passthrough > BPE (if merges) > basic."""
    if passthrough:
        return PassthroughStrategy()
    if bpe_merges is not None:
        return BpeStrategy.new(bpe_merges)
    return BasicTokenizationStrategy()


def run_tokenizer(data, chunk_size: int, strategy: TokenizationStrategy, content_type: Optional[str] = None,
                  n_gpus: int = 1) -> bytes:
    """run_tokenizer over an in-memory buffer (lib.rs:239-265): the optional content-type token
    (lib.rs:284-293), then every chunk of chunk_size bytes (pipeline.rs:73-81) tokenised and
    stitched in chunk order (pipeline.rs:153-192).  BPE runs as one batched GPU call."""
    head = b"" if content_type is None else ContentType.BY_NAME[content_type].to_bytes(2, "big")
    if chunk_size <= 0:
        raise ValueError("chunk_size must be > 0")
    if isinstance(strategy, BpeStrategy):
        import numpy as np
        return head + bytes(np.asarray(strategy.process_chunks(data, chunk_size, n_gpus=n_gpus)))
    mv = memoryview(data).cast("B")
    # basic and passthrough are per byte: the chunk split does not change the stream
    return head + strategy.process_chunk(mv) if len(mv) else head


def file_tokenizer(input_path: Optional[str], output_path: Optional[str], strategy: Optional[TokenizationStrategy],
                   content_type: Optional[int], threads: int, chunk_size: int, n_gpus: int = 0) -> None:
    """run_tokenizer (lib.rs:246-267) over files through the library's pipeline (blt_run_tokenizer):
    input file (mmap, fixed chunks) or stdin when None, output file (created after the input is
    opened) or stdout when None, content-type token, chunks in order.  Raises BltError."""
    cfg = _lib.RunConfig()
    cfg.input_path = None if input_path is None else os.fsencode(input_path)
    cfg.output_path = None if output_path is None else os.fsencode(output_path)
    cfg.passthrough = int(isinstance(strategy, PassthroughStrategy))
    cfg.bpe = strategy.handle if isinstance(strategy, BpeStrategy) else None
    cfg.content_token = content_type or 0
    cfg.threads = max(1, int(threads))
    cfg.chunk_size = int(chunk_size)
    cfg.n_gpus = int(n_gpus)
    _lib.check(_lib.lib().blt_run_tokenizer(ctypes.byref(cfg)))


def _u(value, bits: int, name: str) -> int:
    """PyO3's extraction of a Rust unsigned integer: TypeError for a non-int, OverflowError outside
    the type's range."""
    if isinstance(value, bool) or not isinstance(value, int):
        raise TypeError(f"'{type(value).__name__}' object cannot be interpreted as an integer ({name})")
    if value < 0 or value >= (1 << bits):
        raise OverflowError(f"{name} out of range for u{bits}: {value}")
    return value


def _debug_opt(v) -> str:
    """Rust's {:?} of an Option<String> / Option<int>."""
    if v is None:
        return "None"
    if isinstance(v, str):
        return "Some(" + json.dumps(v) + ")"
    return f"Some({v})"


class ByteTokenizer:
    """ByteTokenizer (blt_python/src/lib.rs:27-170) over the MI355X library.

    ``merges``: {(byte1, byte2): token_id}; ``content_type``: "Text" or "Bin" (the reference
    binding accepts only these two, lib.rs:66-75); ``threads``: chunks in flight; ``chunk_size``:
    e.g. "16MB" (utils.rs:10-45); ``memory_cap``: percent of RAM for the automatic chunk size
    (0-100, lib.rs:57-63).

    Token ids follow the reference binding: it writes the dict's KEYS, one "a b" line each, to a
    temporary merges file and loads that file (lib.rs:103-114, config_loader.rs:14-46), so the ids
    are 256, 257, ... in the order the keys are written and the dict's values are ignored.  The
    reference writes them in HashMap iteration order (random per process); here they are written in
    the dict's insertion order, which is one of the reference's possible outcomes, and the same
    temporary-file load runs (so every loader rule applies, the u16 wrap past 65,280 keys included).
    ``use_dict_ids=True`` (not in the reference) takes the dict's values as the ids instead.
    """

    def __init__(self, merges: Optional[Dict[Tuple[int, int], int]] = None, content_type: Optional[str] = None,
                 threads: Optional[int] = None, chunk_size: Optional[str] = None, memory_cap: Optional[int] = None,
                 *, use_dict_ids: bool = False):
        if merges is not None:
            if not isinstance(merges, dict):
                raise TypeError("merges must be a dict {(byte1, byte2): token_id}")
            merges = {(_u(a, 8, "byte1"), _u(b, 8, "byte2")): _u(v, 16, "token_id") for (a, b), v in merges.items()}
        if threads is not None:
            threads = _u(threads, 64, "threads")
        if memory_cap is not None:
            memory_cap = _u(memory_cap, 8, "memory_cap")
            if memory_cap > 100:   # lib.rs:57-63
                raise ValueError("memory_cap must be between 0 and 100")
        if content_type is not None:
            if not isinstance(content_type, str):
                raise TypeError("content_type must be a string")
            if content_type not in ("Text", "Bin"):   # lib.rs:66-75
                raise ValueError("content_type must be 'Text' or 'Bin'")
        if chunk_size is not None and not isinstance(chunk_size, str):
            raise TypeError("chunk_size must be a string such as '1MB'")
        self._merges = merges
        self._content_type = content_type
        self._threads = threads
        self._chunk_size = chunk_size
        self._memory_cap = memory_cap
        self._use_dict_ids = bool(use_dict_ids)

    def tokenize_file(self, input_path: str, output_path: str) -> None:
        """lib.rs:90-159: CoreConfig::new_from_cli + run_tokenizer on the two files.  Raises OSError
        (BltError) on I/O, configuration or GPU failures."""
        threads = determine_thread_count(self._threads)
        cli_cs = None
        if self._chunk_size is not None:
            out = ctypes.c_uint64(0)
            L = _lib.lib()
            rc = L.blt_parse_chunk_size(self._chunk_size.encode(), ctypes.byref(out))
            if rc:
                raise BltError(rc, L.blt_last_error().decode())   # io::ErrorKind::InvalidInput
            cli_cs = out.value
        mem_cap = 80 if self._memory_cap is None else self._memory_cap   # lib.rs:172
        cs = get_effective_chunk_size(cli_cs, threads, mem_cap)
        strategy = self._strategy()
        token = {"Text": ContentType.Text, "Bin": ContentType.Bin}.get(self._content_type)
        try:
            file_tokenizer(os.fspath(input_path), os.fspath(output_path), strategy, token, threads, cs)
        finally:
            if isinstance(strategy, BpeStrategy):
                strategy.close()

    def _strategy(self) -> TokenizationStrategy:
        if self._merges is None:
            return BasicTokenizationStrategy()
        if self._use_dict_ids:
            return BpeStrategy(self._merges)
        import tempfile
        # lib.rs:103-114: the keys, one "a b" line each, then the file goes through the loader
        fd, path = tempfile.mkstemp(prefix="blt_merges_", suffix=".txt")
        try:
            with os.fdopen(fd, "w") as f:
                f.write("".join(f"{a} {b}\n" for a, b in self._merges))
            return BpeStrategy.from_file(path)
        finally:
            os.unlink(path)

    def __repr__(self) -> str:   # lib.rs:162-170
        return (f"ByteTokenizer(merges={len(self._merges) if self._merges is not None else 0}, "
                f"content_type={_debug_opt(self._content_type)}, threads={_debug_opt(self._threads)}, "
                f"chunk_size={_debug_opt(self._chunk_size)}, memory_cap={_debug_opt(self._memory_cap)})")

    __str__ = __repr__


__version__ = version()
