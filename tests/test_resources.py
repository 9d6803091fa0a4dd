"""Register spills of the product kernels: the kernel source compiled for gfx950
with -Rpass-analysis=kernel-resource-usage (device compile only, ~30 s, no GPU).  A VGPR spill
puts scratch loads and stores, and their vmcnt waits, into the loop of a latency-bound kernel; the
byte pass and the u16 scan kernels sit at the 128-VGPR ceiling of 4 waves per SIMD, so a small
change can push them over.  This test fails as soon as one of them spills a VGPR."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import resources  # noqa: E402

# Kernels on the default paths: every byte-pass instantiation (every merges file, and pass 1 of
# every general map), the u16 scan passes and the fused passes 1 + 2, the finish kernels, the sparse
# passes of cyclic maps, the basic strategy.
DEFAULT_PATH = ("scan_bytes_kernel", "scan_tokens_kernel", "finish_chunks_kernel", "finish_gate_kernel",
                "chunk_map_kernel", "chain_final_kernel", "basic_expand_kernel", "sparse_")


@pytest.fixture(scope="module")
def res():
    return resources.parse(resources.remarks())


def test_every_kernel_reported(res):
    names = " ".join(res)
    for k in DEFAULT_PATH:
        assert k in names, k


def test_no_vgpr_spills_on_default_paths(res):
    bad = {resources.demangle(k): r for k, r in res.items()
           if any(d in k for d in DEFAULT_PATH) and (r.get("vgpr_spill", 0) or r.get("scratch", 0))}
    assert not bad, resources.table(bad)


def test_byte_pass_occupancy(res):
    """The byte pass keeps 4 waves per SIMD (one 1024-thread workgroup per CU, 128 VGPRs)."""
    for k, r in res.items():
        if "scan_bytes_kernel" in k:
            assert r["waves"] == 4 and r["vgprs"] <= 128, (resources.demangle(k), r)
