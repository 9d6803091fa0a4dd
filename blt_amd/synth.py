"""Seeded synthetic workloads of SURVEY.md §8(d) / BASELINE.json configs (bench and tests).

* ``text(n, seed, offset=0)``   — English-like text: words over a-z with English letter
  frequencies, geometric length 1-12, separated by ' ' or (p = 1/12) '\\n'.
* ``random_bytes(n, seed, offset=0)`` — uniform random bytes.
* ``top_pair_merges(data, k)`` — the k most frequent adjacent byte pairs (ties by pair value),
  as merges-file lines: cfg2 uses k = 256.
* ``text_merges_50k(data, seed)`` — every pair seen in the text by frequency, then the remaining
  pairs in a seeded permutation, up to 50 000 lines (cfg3/cfg4/cfg5).
* General maps of SURVEY.md §8 row f2 (several passes, tokenizer.rs:63-86): ``CHAINED_TEXT_MAP``
  (chained and byte-valued merges on text), ``SELF_VALUED_MAP`` (merges whose value is their own
  first byte, which only the generic byte pass takes), ``doubling_chain(depth)`` (one pass per
  level over runs of one byte), ``wrap_merges_lines()`` (a 65 537-line merges file whose u16 ids
  wrap, config_loader.rs:18, :40).

Streams are generated in independent 1 MiB blocks, so ``offset`` selects any slice of a longer
stream (each rank of a multi-GPU run generates only its shard).
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, List, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def _load():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, "libblt_synth.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} is not built: run `make`")
        L = ctypes.CDLL(path)
        for f in (L.blt_synth_text, L.blt_synth_random):
            f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_uint64]
            f.restype = None
        L.blt_synth_pair_counts.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.blt_synth_pair_counts.restype = None
        _lib = L
    return _lib


def text(n: int, seed: int, offset: int = 0, out: np.ndarray = None) -> np.ndarray:
    a = np.empty(n, dtype=np.uint8) if out is None else out
    _load().blt_synth_text(a.ctypes.data, offset, n, seed)
    return a


def random_bytes(n: int, seed: int, offset: int = 0, out: np.ndarray = None) -> np.ndarray:
    a = np.empty(n, dtype=np.uint8) if out is None else out
    _load().blt_synth_random(a.ctypes.data, offset, n, seed)
    return a


def pair_counts(data: np.ndarray) -> np.ndarray:
    c = np.zeros(65536, dtype=np.uint64)
    d = np.ascontiguousarray(data, dtype=np.uint8)
    _load().blt_synth_pair_counts(d.ctypes.data, d.size, c.ctypes.data)
    return c


def _rank(counts: np.ndarray) -> np.ndarray:
    """Pair values with count > 0, by count descending then pair value ascending."""
    idx = np.nonzero(counts)[0]
    order = np.lexsort((idx, -counts[idx].astype(np.int64)))
    return idx[order]


def top_pair_merges(data: np.ndarray, k: int = 256) -> List[Tuple[int, int]]:
    r = _rank(pair_counts(data))[:k]
    return [(int(p) >> 8, int(p) & 255) for p in r]


def text_merges_50k(data: np.ndarray, seed: int, total: int = 50000) -> List[Tuple[int, int]]:
    seen = _rank(pair_counts(data))
    mask = np.ones(65536, dtype=bool)
    mask[seen] = False
    rest = np.nonzero(mask)[0]
    rng = np.random.default_rng(seed)
    rest = rest[rng.permutation(rest.size)]
    allp = np.concatenate([seen, rest])[:total]
    return [(int(p) >> 8, int(p) & 255) for p in allp]


def merges_file_text(pairs: List[Tuple[int, int]]) -> str:
    return "".join(f"{a} {b}\n" for a, b in pairs)


def merges_dict(pairs: List[Tuple[int, int]]) -> Dict[Tuple[int, int], int]:
    """The map a merges file with these lines loads to (config_loader.rs:39-40)."""
    d: Dict[Tuple[int, int], int] = {}
    for i, (a, b) in enumerate(pairs):
        d[(a, b)] = (256 + i) & 0xFFFF
    return d


# f2 workloads (general maps: a byte pass, then u16 passes until one merges nothing)
CHAINED_TEXT_MAP = {(101, 32): 256, (256, 116): 257, (116, 104): 65, (65, 101): 258, (32, 116): 259, (259, 104): 260}
# "e " -> e and "th" -> t (value = its own first byte: the self-token byte kernel cannot take it),
# "in" -> 256, then "in" "g" -> 257
SELF_VALUED_MAP = {(101, 32): 101, (116, 104): 116, (105, 110): 256, (256, 103): 257}


def doubling_chain(depth: int) -> Dict[Tuple[int, int], int]:
    """(97, 97) -> 256, (256, 256) -> 257, ...: a run of 2^depth 'a' is one token after depth passes."""
    m = {(97, 97): 256}
    for k in range(1, depth):
        m[(255 + k, 255 + k)] = 256 + k
    return m


def wrap_merges_lines() -> str:
    """Every byte pair in order, then "1 2": 65 537 lines; ids wrap to 0..255 after line 65 280."""
    return "".join(f"{i >> 8} {i & 255}\n" for i in range(65536)) + "1 2\n"
