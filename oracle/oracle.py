"""ORACLE — TEST INFRASTRUCTURE ONLY.  NOT PART OF THE PRODUCT PATH.

Two CPU restatements of the reference's BPE merge-scan path (jtrefon/blt, Rust):

* pure-Python functions (``bpe_process_chunk`` …) for small cases, written straight from the
  reference source, and
* ctypes bindings to the plain-C restatement in ``bpe_oracle.c`` (``COracle``) for large
  inputs and the CPU baseline.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import this
module, and only as the checker.  The GPU product never calls it.

Parity: the reference cannot run here (no Rust toolchain).  Both restatements are pinned by
the reference's own known-answer tests, transcribed as data into
``tests/golden/reference_kats.json`` (see tests/test_oracle_kats.py).
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

_HERE = os.path.dirname(os.path.abspath(__file__))

CONTENT_TOKENS = {"text": 0xFF01, "audio": 0xFF02, "bin": 0xFF03, "video": 0xFF04}  # lib.rs:93-104


# ----------------------------------------------------------------------------------------
# Pure-Python restatement
# ----------------------------------------------------------------------------------------
def bpe_process_chunk(merges: Dict[Tuple[int, int], int], chunk: bytes) -> bytes:
    """BpeStrategy::process_chunk — blt_core/src/tokenizer.rs:56-93."""
    if len(chunk) == 0:  # :57-59
        return b""
    tokens = list(chunk)  # :61 widen u8 -> u16
    while True:  # :63
        merges_found = False
        new_tokens = []
        i = 0
        while i < len(tokens):  # :67
            if i < len(tokens) - 1:
                v = merges.get((tokens[i], tokens[i + 1]))
                if v is not None:  # :69-72
                    new_tokens.append(v)
                    i += 2
                    merges_found = True
                else:  # :73-76
                    new_tokens.append(tokens[i])
                    i += 1
            else:  # :77-80
                new_tokens.append(tokens[i])
                i += 1
        tokens = new_tokens
        if not merges_found:  # :83-85
            break
    out = bytearray()
    for t in tokens:  # :88-91 big-endian u16
        out += bytes(((t >> 8) & 0xFF, t & 0xFF))
    return bytes(out)


def basic_process_chunk(chunk: bytes) -> bytes:
    """BasicTokenizationStrategy::process_chunk — tokenizer.rs:108-124."""
    out = bytearray(2 * len(chunk))
    out[1::2] = chunk
    return bytes(out)


def passthrough_process_chunk(chunk: bytes) -> bytes:
    """PassthroughStrategy::process_chunk — tokenizer.rs:138-144."""
    return bytes(chunk)


def split_chunks(n: int, chunk_size: int) -> List[Tuple[int, int]]:
    """mmap.chunks(cs) — blt_core/src/pipeline.rs:73-81: (start, len) per chunk."""
    return [(s, min(chunk_size, n - s)) for s in range(0, n, chunk_size)]


def run_chunks(data: bytes, chunk_size: int, merges: Optional[Dict] = None, passthrough: bool = False,
               content_type: Optional[str] = None) -> bytes:
    """run_tokenizer's mmap path: select_strategy (lib.rs:271-282), content token
    (lib.rs:284-293), chunk split (pipeline.rs:73-81), ordered stitch (pipeline.rs:153-192)."""
    out = bytearray()
    if content_type is not None:
        out += CONTENT_TOKENS[content_type].to_bytes(2, "big")
    for s, ln in split_chunks(len(data), chunk_size):
        c = data[s:s + ln]
        if passthrough:
            out += passthrough_process_chunk(c)
        elif merges is not None:
            out += bpe_process_chunk(merges, c)
        else:
            out += basic_process_chunk(c)
    return bytes(out)


class MergeLoadError(Exception):
    """io::Error from load_bpe_merges_from_path: kind in {'NotFound', 'InvalidData', 'Other'}."""

    def __init__(self, kind: str, message: str):
        super().__init__(message)
        self.kind = kind


_WS = {0x09, 0x0A, 0x0B, 0x0C, 0x0D, 0x20, 0x85, 0xA0, 0x1680, 0x2028, 0x2029, 0x202F, 0x205F,
       0x3000} | set(range(0x2000, 0x200B))


def _split_whitespace(s: str) -> List[str]:
    """str::split_whitespace (Unicode White_Space)."""
    parts, cur = [], []
    for ch in s:
        if ord(ch) in _WS:
            if cur:
                parts.append("".join(cur))
                cur = []
        else:
            cur.append(ch)
    if cur:
        parts.append("".join(cur))
    return parts


def _parse_uint(s: str, limit: int) -> Tuple[Optional[int], Optional[str]]:
    """<uN as FromStr>::from_str, radix 10 (core::num): optional '+', ASCII digits; the digit
    check precedes the overflow report for each char."""
    if s == "":
        return None, "cannot parse integer from empty string"
    i = 0
    if s[0] in "+-":
        if len(s) == 1:
            return None, "invalid digit found in string"
        if s[0] == "+":
            i = 1
    r = 0
    for ch in s[i:]:
        mul_ok = r * 10 <= limit
        if not ("0" <= ch <= "9"):
            return None, "invalid digit found in string"
        if not mul_ok:
            return None, "number too large to fit in target type"
        r = r * 10 + (ord(ch) - 48)
        if r > limit:
            return None, "number too large to fit in target type"
    return r, None


def load_bpe_merges_from_path(path: str) -> Dict[Tuple[int, int], int]:
    """load_bpe_merges_from_path — blt_core/src/config_loader.rs:14-46 (release-build u16 wrap)."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except FileNotFoundError as e:
        raise MergeLoadError("NotFound", f"{os.strerror(e.errno)} (os error {e.errno})")
    except OSError as e:
        raise MergeLoadError("Other", f"{os.strerror(e.errno)} (os error {e.errno})")
    merges: Dict[Tuple[int, int], int] = {}
    vocab = 256  # :18
    pos = 0
    while pos < len(data):  # BufRead::lines
        e = data.find(b"\n", pos)
        had_nl = e >= 0
        if not had_nl:
            e = len(data)
        line_b = data[pos:e]
        consumed = data[pos:e + 1] if had_nl else line_b
        pos = e + 1 if had_nl else e
        try:  # read_line validates the appended bytes
            consumed.decode("utf-8")
        except UnicodeDecodeError:
            raise MergeLoadError("InvalidData", "stream did not contain valid UTF-8")
        if had_nl and line_b.endswith(b"\r"):  # lines() pops "\n" then "\r"
            line_b = line_b[:-1]
        line = line_b.decode("utf-8")
        if line.startswith("#") or line == "":  # :22
            continue
        parts = _split_whitespace(line)  # :25
        if len(parts) != 2:  # :41-43
            raise MergeLoadError(
                "InvalidData",
                f"Invalid merge rule format in line: '{line}'. Expected two numbers separated by space.")
        b1, err = _parse_uint(parts[0], 255)
        if err:
            raise MergeLoadError("InvalidData", f"Failed to parse first byte value: {err} in line '{line}'")
        b2, err = _parse_uint(parts[1], 255)
        if err:
            raise MergeLoadError("InvalidData", f"Failed to parse second byte value: {err} in line '{line}'")
        merges[(b1, b2)] = vocab  # :39
        vocab = (vocab + 1) & 0xFFFF  # :40 (u16 wraps: no overflow-checks in release)
    return merges


def parse_chunk_size_str(s: str) -> int:
    """parse_chunk_size_str — blt_core/src/utils.rs:10-45.  Raises ValueError(msg)."""
    t = s.strip("".join(chr(c) for c in _WS))
    if t == "":
        raise ValueError("Input string is empty")
    up = t.upper()
    if up.endswith("KB") or up.endswith("MB"):
        num, unit = t[:-2], t[-2:]
    elif all("0" <= c <= "9" for c in up):
        num, unit = t, ""
    else:
        raise ValueError(f"Invalid unit or format: '{t}'. Number must be followed by KB, MB, or be raw bytes.")
    if num == "" and unit != "":
        raise ValueError(f"Number part missing for unit '{unit}'")
    v, err = _parse_uint(num, (1 << 64) - 1)
    if err:
        raise ValueError(f"Invalid number: '{num}'")
    mult = {"KB": 1024, "MB": 1024 * 1024, "": 1}[unit.upper()]
    return (v * mult) & ((1 << 64) - 1)  # release-build wrapping multiply


ABSOLUTE_MIN_CHUNK_SIZE = 256 * 1024  # chunking.rs:17-20
ABSOLUTE_MAX_CHUNK_SIZE = 128 * 1024 * 1024
DEFAULT_MIN_CHUNK_SIZE_BYTES = 1024 * 1024
DEFAULT_MAX_CHUNK_SIZE_BYTES = 16 * 1024 * 1024


def get_effective_chunk_size(cli_chunk_size: Optional[int], num_threads: int, mem_cap_percent: int,
                             total_ram_bytes: int) -> int:
    """get_effective_chunk_size — blt_core/src/chunking.rs:26-62."""
    if cli_chunk_size is not None:
        return min(max(cli_chunk_size, ABSOLUTE_MIN_CHUNK_SIZE), ABSOLUTE_MAX_CHUNK_SIZE)
    usable = int(float(total_ram_bytes) * (float(mem_cap_percent) / 100.0))
    c = (usable // num_threads) // 4
    c = min(max(c, DEFAULT_MIN_CHUNK_SIZE_BYTES), DEFAULT_MAX_CHUNK_SIZE_BYTES)
    return min(max(c, ABSOLUTE_MIN_CHUNK_SIZE), ABSOLUTE_MAX_CHUNK_SIZE)


def determine_thread_count(threads: Optional[int]) -> int:
    """determine_thread_count — blt_core/src/utils.rs:79-97."""
    if threads is not None:
        return 1 if threads == 0 else threads
    return max(1, os.cpu_count() or 1)


# ----------------------------------------------------------------------------------------
# ctypes binding to the C restatement (bpe_oracle.c)
# ----------------------------------------------------------------------------------------
_lib = None


def _load():
    global _lib
    if _lib is not None:
        return _lib
    path = os.path.join(_HERE, "liboracle.so")
    if not os.path.exists(path):
        raise RuntimeError(f"oracle library not built: {path} (run `make -C oracle`)")
    lib = ctypes.CDLL(path)
    u16p = ctypes.POINTER(ctypes.c_uint16)
    lib.oracle_map_new.restype = ctypes.c_void_p
    lib.oracle_map_new.argtypes = [u16p, u16p, u16p, ctypes.c_size_t]
    lib.oracle_map_free.argtypes = [ctypes.c_void_p]
    lib.oracle_bpe_process_chunk.restype = ctypes.c_size_t
    lib.oracle_bpe_process_chunk.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    lib.oracle_run_chunks.restype = ctypes.c_size_t
    lib.oracle_run_chunks.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_void_p]
    lib.oracle_fast_run_chunks.restype = ctypes.c_size_t
    lib.oracle_fast_run_chunks.argtypes = [u16p, u16p, u16p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    lib.oracle_load_merges.restype = ctypes.c_int
    lib.oracle_load_merges.argtypes = [ctypes.c_char_p, u16p, u16p, u16p, ctypes.c_size_t,
                                       ctypes.POINTER(ctypes.c_size_t), ctypes.c_char_p, ctypes.c_size_t]
    lib.oracle_parse_chunk_size.restype = ctypes.c_int
    lib.oracle_parse_chunk_size.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64),
                                            ctypes.c_char_p, ctypes.c_size_t]
    lib.oracle_effective_chunk_size.restype = ctypes.c_uint64
    lib.oracle_effective_chunk_size.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                                ctypes.c_uint, ctypes.c_uint64]
    _lib = lib
    return lib


def _as_buffer(data):
    """Returns (pointer, keepalive) for bytes / bytearray / numpy uint8 arrays."""
    try:
        import numpy as np
        if isinstance(data, np.ndarray):
            a = np.ascontiguousarray(data, dtype=np.uint8)
            return a.ctypes.data, a
    except ImportError:  # pragma: no cover
        pass
    b = (ctypes.c_uint8 * len(data)).from_buffer_copy(bytes(data)) if len(data) else (ctypes.c_uint8 * 1)()
    return ctypes.addressof(b), b


class COracle:
    """The C restatement of BpeStrategy over an arbitrary BpeMerges map (tokenizer.rs:56-93)."""

    def __init__(self, merges: Optional[Dict[Tuple[int, int], int]]):
        self._lib = _load()
        self._map = None
        if merges is not None:
            items = list(merges.items())
            n = len(items)
            A = (ctypes.c_uint16 * max(n, 1))(*[k[0] for k, _ in items])
            B = (ctypes.c_uint16 * max(n, 1))(*[k[1] for k, _ in items])
            V = (ctypes.c_uint16 * max(n, 1))(*[v for _, v in items])
            self._map = self._lib.oracle_map_new(A, B, V, n)

    def __del__(self):
        if getattr(self, "_map", None):
            self._lib.oracle_map_free(self._map)
            self._map = None

    def process_chunk(self, chunk) -> bytes:
        ptr, keep = _as_buffer(chunk)
        n = len(chunk)
        out = (ctypes.c_uint8 * max(2 * n, 1))()
        if self._map is None:
            return self.run(chunk, max(n, 1), threads=1)
        m = self._lib.oracle_bpe_process_chunk(self._map, ptr, n, out)
        return bytes(out[:m])

    def run(self, data, chunk_size: int, content_type: Optional[str] = None, threads: int = 1,
            passthrough: bool = False, return_lens: bool = False):
        import numpy as np
        ptr, keep = _as_buffer(data)
        n = len(data)
        out = np.empty(2 * n + 2, dtype=np.uint8)
        nchunks = (n + chunk_size - 1) // chunk_size if n else 0
        lens = np.zeros(max(nchunks, 1), dtype=np.uint64)
        tok = CONTENT_TOKENS[content_type] if content_type else -1
        m = self._lib.oracle_run_chunks(self._map, int(passthrough), ptr, n, chunk_size, tok, threads,
                                        out.ctypes.data, lens.ctypes.data)
        res = out[:m]
        if return_lens:
            return res, lens[:nchunks].astype(np.int64)
        return res


def fast_run(merges: Dict[Tuple[int, int], int], data, chunk_size: int, threads: int = 1):
    """The "optimised CPU" line: dense table, one greedy pass per chunk, for a
    single-pass byte-pair map.  A baseline for bench.py, never a checker.  Returns None for maps
    it does not cover (u16 keys, or a value that is a key component)."""
    import numpy as np
    lib = _load()
    items = list(merges.items())
    nm = len(items)
    A = (ctypes.c_uint16 * max(nm, 1))(*[k[0] for k, _ in items])
    B = (ctypes.c_uint16 * max(nm, 1))(*[k[1] for k, _ in items])
    V = (ctypes.c_uint16 * max(nm, 1))(*[v for _, v in items])
    ptr, keep = _as_buffer(data)
    n = len(data)
    out = np.empty(max(2 * n, 1), dtype=np.uint8)
    m = lib.oracle_fast_run_chunks(A, B, V, nm, ptr, n, chunk_size, threads, out.ctypes.data)
    if m == ctypes.c_size_t(-1).value:
        return None
    return out[:m]


def c_load_merges(path: str) -> Dict[Tuple[int, int], int]:
    lib = _load()
    cap = 65536
    A = (ctypes.c_uint16 * cap)()
    B = (ctypes.c_uint16 * cap)()
    V = (ctypes.c_uint16 * cap)()
    n = ctypes.c_size_t(0)
    msg = ctypes.create_string_buffer(4096)
    rc = lib.oracle_load_merges(path.encode(), A, B, V, cap, ctypes.byref(n), msg, 4096)
    if rc != 0:
        kind = {1: "NotFound", 2: "InvalidData"}.get(rc, "Other")
        raise MergeLoadError(kind, msg.value.decode("utf-8", "replace"))
    return {(A[i], B[i]): V[i] for i in range(n.value)}


def c_parse_chunk_size(s: str) -> int:
    lib = _load()
    out = ctypes.c_uint64(0)
    msg = ctypes.create_string_buffer(1024)
    if lib.oracle_parse_chunk_size(s.encode(), ctypes.byref(out), msg, 1024) != 0:
        raise ValueError(msg.value.decode())
    return out.value


def c_effective_chunk_size(cli: Optional[int], threads: int, memcap: int, total_ram: int) -> int:
    lib = _load()
    return lib.oracle_effective_chunk_size(int(cli is not None), cli or 0, threads, memcap, total_ram)
