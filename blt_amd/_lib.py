"""ctypes binding of include/blt_bpe.h (libblt_bpe.so, built in-tree by `make`).

The library is the product: HIP kernels for gfx950 plus the C ABI.  Loading it needs no GPU;
every tokenising call does, and fails loudly (BLT_E_NODEV) without one — there is no CPU path.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# BLT_LIB_PATH: an alternative build of the same library (tools/ timing experiments only).
LIB_PATH = os.environ.get("BLT_LIB_PATH") or os.path.join(_HERE, "libblt_bpe.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "blt_bpe.h")

BLT_E_NOT_FOUND = -2
BLT_E_INVALID_DATA = -74
BLT_E_INVALID_INPUT = -22
BLT_E_NOSPC = -28
BLT_E_NOMEM = -12
BLT_E_IO = -5
BLT_E_NODEV = -19

ERROR_KINDS = {
    BLT_E_NOT_FOUND: "NotFound",
    BLT_E_INVALID_DATA: "InvalidData",
    BLT_E_INVALID_INPUT: "InvalidInput",
    BLT_E_NOSPC: "NoSpace",
    BLT_E_NOMEM: "OutOfMemory",
    BLT_E_IO: "Other",
    BLT_E_NODEV: "NoDevice",
}


class BltError(OSError):
    """A failing C-ABI call: .code is the negative errno, .kind the reference io::ErrorKind."""

    def __init__(self, code: int, message: str):
        super().__init__(-code, message)
        self.code = code
        self.kind = ERROR_KINDS.get(code, "Other")
        self.message = message

    def __str__(self):
        return self.message


_lib = None

_u16p = ctypes.POINTER(ctypes.c_uint16)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_szp = ctypes.POINTER(ctypes.c_size_t)
_vp = ctypes.c_void_p

class RunConfig(ctypes.Structure):
    """blt_run_config (include/blt_bpe.h)."""
    _fields_ = [("input_path", ctypes.c_char_p), ("output_path", ctypes.c_char_p), ("bpe", ctypes.c_void_p),
                ("passthrough", ctypes.c_int), ("content_token", ctypes.c_uint32), ("threads", ctypes.c_uint64),
                ("chunk_size", ctypes.c_uint64), ("n_gpus", ctypes.c_int)]


_SIGNATURES = {
    "blt_version": (ctypes.c_char_p, []),
    "blt_last_error": (ctypes.c_char_p, []),
    "blt_load_bpe_merges": (ctypes.c_int, [ctypes.c_char_p, _u16p, _u16p, _u16p, ctypes.c_size_t, _szp]),
    "blt_parse_chunk_size": (ctypes.c_int, [ctypes.c_char_p, _u64p]),
    "blt_effective_chunk_size": (ctypes.c_uint64, [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]),
    "blt_determine_thread_count": (ctypes.c_uint64, [ctypes.c_int, ctypes.c_uint64]),
    "blt_bpe_create": (ctypes.c_int, [_u16p, _u16p, _u16p, ctypes.c_size_t, ctypes.c_uint32, ctypes.POINTER(_vp)]),
    "blt_bpe_create_from_file": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(_vp)]),
    "blt_bpe_destroy": (None, [_vp]),
    "blt_bpe_info": (ctypes.c_int, [_vp, _szp, ctypes.POINTER(ctypes.c_int)]),
    "blt_bpe_clear_error": (ctypes.c_int, [_vp]),
    "blt_run_tokenizer": (ctypes.c_int, [ctypes.POINTER(RunConfig)]),
    "blt_bpe_process_chunk": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, _vp, ctypes.c_size_t, _szp]),
    "blt_bpe_process_chunks": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, _vp,
                                              ctypes.c_size_t, _szp, _vp]),
    "blt_basic_process_chunk": (ctypes.c_int, [_vp, ctypes.c_size_t, _vp, ctypes.c_size_t, _szp]),
    "blt_bpe_workspace_size": (ctypes.c_size_t, [_vp, ctypes.c_uint64, ctypes.c_uint64]),
    "blt_bpe_encode_device": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_uint64, _vp, _vp, _vp,
                                             ctypes.c_size_t, _vp, _u64p]),
    "blt_bpe_encode_device_ex": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_uint64, _vp, _vp, _vp,
                                                ctypes.c_size_t, _vp, _u64p, ctypes.c_uint32]),
    "blt_bpe_workspace_reset": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_uint64, _vp]),
    "blt_bpe_check_workspace": (ctypes.c_int, [_vp, _vp]),
    "blt_basic_encode_device": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, _vp]),
}

# Test hooks exported by the library but not declared in the header.
_DEBUG_SIGNATURES = {
    "blt_debug_inject_device_error": (ctypes.c_int, [_vp, _vp, _vp]),
    "blt_debug_set_tile_record": (None, [_vp]),
    "blt_debug_set_inject": (ctypes.c_uint32, [ctypes.c_uint32]),
    "blt_debug_last_u16_passes": (ctypes.c_uint32, []),
    "blt_debug_last_scan_passes": (ctypes.c_uint32, []),
    "blt_debug_set_u16_chain": (ctypes.c_int, [ctypes.c_int]),
    "blt_debug_set_fused_only": (ctypes.c_int, [ctypes.c_int]),
    "blt_debug_set_shared_contexts": (None, [ctypes.c_int]),
    "blt_debug_set_pin_ring": (ctypes.c_int, [ctypes.c_int]),
    "blt_debug_set_fused": (None, [ctypes.c_int]),
    "blt_debug_last_fused": (ctypes.c_uint32, []),
    "blt_debug_byte_mode": (ctypes.c_int, [_vp]),
    "blt_debug_chain_depth": (ctypes.c_uint32, [_vp]),
    "blt_debug_set_finish": (ctypes.c_int, [ctypes.c_int]),
    "blt_debug_set_sparse": (ctypes.c_int, [ctypes.c_int]),
    "blt_debug_last_sparse": (ctypes.c_uint32, []),
    "blt_debug_set_sparse_cap": (ctypes.c_uint32, [ctypes.c_uint32]),
    "blt_debug_available_cpus": (ctypes.c_uint64, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64]),
}


def header_symbols():
    """Function names declared in include/blt_bpe.h."""
    with open(HEADER_PATH) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(blt_[a-z0-9_]+)\s*\(", text)))


def _share_torch_runtime():
    """PyTorch-ROCm wheels bundle their own libamdhip64.so with the same SONAME
    (libamdhip64.so.7) as /opt/rocm's.  Loading torch's copy first makes our library's
    DT_NEEDED resolve to it, so a process that also uses torch has ONE HIP runtime; loading
    ours first would make torch load a second runtime, which then finds no GPU."""
    if os.environ.get("BLT_STANDALONE_HIP") == "1":
        return
    try:
        import torch  # noqa: F401
        import torch.cuda  # noqa: F401
        libdir = os.path.join(os.path.dirname(torch.__file__), "lib")
        hip = os.path.join(libdir, "libamdhip64.so")
        if os.path.exists(hip):
            ctypes.CDLL(hip, mode=ctypes.RTLD_GLOBAL)
    except ImportError:
        pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is not built: run `make` (or __graft_entry__.build())")
        _share_torch_runtime()
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in list(_SIGNATURES.items()) + list(_DEBUG_SIGNATURES.items()):
            try:
                fn = getattr(L, name)
            except AttributeError:
                if name in _DEBUG_SIGNATURES:   # test hooks an older experiment build may lack
                    continue
                raise
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != 0:
        msg = lib().blt_last_error().decode("utf-8", "replace")
        raise BltError(rc, msg)
