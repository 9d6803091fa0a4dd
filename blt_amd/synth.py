"""Seeded synthetic workloads of SURVEY.md §8(d) / BASELINE.json configs (bench and tests).

* ``text(n, seed, offset=0)``   — English-like text: words over a-z with English letter
  frequencies, geometric length 1-12, separated by ' ' or (p = 1/12) '\\n'.
* ``random_bytes(n, seed, offset=0)`` — uniform random bytes.
* ``top_pair_merges(data, k)`` — the k most frequent adjacent byte pairs (ties by pair value),
  as merges-file lines: cfg2 uses k = 256.
* ``text_merges_50k(data, seed)`` — every pair seen in the text by frequency, then the remaining
  pairs in a seeded permutation, up to 50 000 lines (cfg3/cfg4/cfg5).

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
