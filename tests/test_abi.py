"""CPU-side checks of the C ABI library: it loads without a GPU, exports every symbol the header
declares, and its host-only functions (merges loader, chunk-size parsing, chunk sizing) agree
with the reference KATs and the oracle, including the loader's edge semantics."""
import ctypes
import os

import pytest

import blt_amd
from blt_amd import _lib
from oracle import oracle as O
from tests.conftest import merges_dict


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    syms = _lib.header_symbols()
    assert len(syms) >= 17
    for s in syms:
        assert hasattr(L, s), s
    assert L.blt_version().decode().startswith("blt-mi355x ")
    assert L.blt_version().decode().split()[-1] == blt_amd.version()


def test_loader_kats(kats, tmp_path):
    for c in kats["loader"]:
        if c["file"] is None:
            path = str(tmp_path / "this_file_should_not_exist.txt")
        else:
            path = str(tmp_path / (c["name"] + ".txt"))
            with open(path, "w") as f:
                f.write(c["file"])
        if "error_kind" in c:
            with pytest.raises(blt_amd.BltError) as ei:
                blt_amd.load_bpe_merges_from_path(path)
            assert ei.value.kind == c["error_kind"], c["name"]
            if "error_contains" in c:
                assert c["error_contains"] in str(ei.value), c["name"]
        else:
            assert blt_amd.load_bpe_merges_from_path(path) == merges_dict(c["merges"]), c["name"]


LOADER_EDGE_FILES = [
    "97 98\r\n99 100\r\n",            # CRLF endings
    "97 98\n\n\n99 100",              # blank lines, no final newline
    "+97 0098\n",                     # '+' sign and leading zeros accepted by u8::from_str
    "97\t98\n",                       # any Unicode whitespace separates fields
    "97 98\n",                   # NBSP is White_Space
    " # x\n",                         # '#' not first: two fields that fail to parse
    "97 98 # ab\n",                   # inline comment: four fields
    "97 98\n97 98\n",                 # duplicate overwrites, counter advances
    "97 -1\n",                        # sign on unsigned
    "97 +\n",                         # bare sign
    "2560 1\n",                       # overflow at the fourth digit
    "25a6 1\n",                       # invalid digit before overflow
    "97 98\r",                        # lone CR at EOF stays in the line (still whitespace)
    "\r\n",                           # CRLF-only line is empty
    "#\n97 98\n",
]


@pytest.mark.parametrize("text", LOADER_EDGE_FILES)
def test_loader_edge_semantics_match_oracle(tmp_path, text):
    path = str(tmp_path / "m.txt")
    with open(path, "w", newline="") as f:
        f.write(text)
    try:
        exp = O.load_bpe_merges_from_path(path)
        exp_err = None
    except O.MergeLoadError as e:
        exp, exp_err = None, (e.kind, str(e))
    try:
        got = blt_amd.load_bpe_merges_from_path(path)
        got_err = None
    except blt_amd.BltError as e:
        got, got_err = None, (e.kind, str(e))
    assert got == exp
    assert got_err == exp_err
    # the C restatement agrees too
    try:
        cexp = O.c_load_merges(path)
        cerr = None
    except O.MergeLoadError as e:
        cexp, cerr = None, (e.kind, str(e))
    assert (cexp, cerr) == (exp, exp_err)


def test_loader_invalid_utf8(tmp_path):
    path = str(tmp_path / "bad.txt")
    with open(path, "wb") as f:
        f.write(b"97 98\n\xff\xfe 1\n")
    with pytest.raises(blt_amd.BltError) as ei:
        blt_amd.load_bpe_merges_from_path(path)
    assert ei.value.kind == "InvalidData"
    assert "valid UTF-8" in str(ei.value)


def test_loader_u16_wrap(tmp_path):
    """65 281 valid lines: the u16 id counter wraps to 0 (release build, config_loader.rs:40)."""
    path = str(tmp_path / "wrap.txt")
    lines = [f"{(i >> 8) & 255} {i & 255}\n" for i in range(65536)] + ["1 2\n"]
    with open(path, "w") as f:
        f.write("".join(lines))
    got = blt_amd.load_bpe_merges_from_path(path)
    exp = O.load_bpe_merges_from_path(path)
    assert got == exp
    assert got[(0, 0)] == 256 and got[(255, 0)] == 0 and got[(1, 2)] == (256 + 65536) & 0xFFFF


def test_parse_chunk_size(kats):
    for c in kats["parse_chunk_size_valid"]:
        assert blt_amd.parse_chunk_size_str(c["s"]) == c["expected"]
    for c in kats["parse_chunk_size_invalid"]:
        with pytest.raises(ValueError):
            blt_amd.parse_chunk_size_str(c["s"])
    for s in ["+5MB", "16MB", "0", "0KB", "18446744073709551615", "99999999999999MB", " 7kB\t", "5 MB", "+5",
              "mb", "1.0", "　1KB　"]:
        try:
            exp = O.parse_chunk_size_str(s)
        except ValueError as e:
            with pytest.raises(ValueError) as ei:
                blt_amd.parse_chunk_size_str(s)
            assert str(ei.value) == str(e)
            continue
        assert blt_amd.parse_chunk_size_str(s) == exp


def test_effective_chunk_size(kats):
    for c in kats["chunk_size_cli"]:
        assert blt_amd.get_effective_chunk_size(c["cli"], c["threads"], c["memcap"]) == c["expected"]
    for c in kats["chunk_size_dynamic_bounds"]:
        v = blt_amd.get_effective_chunk_size(None, c["threads"], c["memcap"])
        assert c["min"] <= v <= c["max"]


def test_thread_count(kats):
    for c in kats["thread_count"]:
        assert blt_amd.determine_thread_count(c["threads"]) == c["expected"]
    assert blt_amd.determine_thread_count(None) >= 1


def _cpus(root, proc, logical):
    return _lib.lib().blt_debug_available_cpus(str(root).encode(), str(proc).encode(), logical)


def test_available_cpus_fake_cgroups(tmp_path):
    """num_cpus::get() (utils.rs:79-97 calls it): min(cgroup quota, logical CPUs) with a quota
    (num_cpus 1.17 init_cgroups, restated: the crate is not vendored), else the logical CPUs."""
    proc = tmp_path / "proc_cgroup"
    proc.write_text("0::/job\n")
    v2 = tmp_path / "v2"
    (v2 / "job").mkdir(parents=True)
    (v2 / "job" / "cpu.max").write_text("1600000 100000\n")   # quota 16 CPUs
    assert _cpus(v2, proc, 256) == 16                           # quota below the affinity mask
    assert _cpus(v2, proc, 8) == 8                              # quota above it: capped
    (v2 / "job" / "cpu.max").write_text("150000 100000\n")     # 1.5 CPUs: ceil
    assert _cpus(v2, proc, 64) == 2
    (v2 / "job" / "cpu.max").write_text("max 100000\n")        # no quota
    assert _cpus(v2, proc, 64) == 64
    v1 = tmp_path / "v1"
    (v1 / "cpu").mkdir(parents=True)
    (v1 / "cpu" / "cpu.cfs_quota_us").write_text("400000\n")
    (v1 / "cpu" / "cpu.cfs_period_us").write_text("100000\n")
    assert _cpus(v1, tmp_path / "missing", 12) == 4
    assert _cpus(v1, tmp_path / "missing", 3) == 3
    (v1 / "cpu" / "cpu.cfs_quota_us").write_text("-1\n")
    assert _cpus(v1, tmp_path / "missing", 12) == 12
    assert _cpus(tmp_path / "none", tmp_path / "missing", 5) == 5


def test_strategy_handle_info():
    s = blt_amd.BpeStrategy({(97, 98): 256, (99, 100): 257})
    assert s.info() == (2, True)
    s2 = blt_amd.BpeStrategy({(97, 98): 256, (256, 99): 257})     # chained: multi-pass
    assert s2.info() == (2, False)
    s3 = blt_amd.BpeStrategy({(120, 121): 90})                      # byte-valued: 90 is not a key part
    assert s3.info() == (1, True)
    s4 = blt_amd.BpeStrategy({(97, 98): 256, (97, 98): 300})
    assert s4.info()[0] == 1


def test_tokenising_without_gpu_fails_loudly():
    """No CPU fallback: with no device the strategy raises BLT_E_NODEV (only meaningful here)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    s = blt_amd.BpeStrategy({(97, 98): 256})
    with pytest.raises(blt_amd.BltError) as ei:
        s.process_chunk(b"abab")
    assert ei.value.kind == "NoDevice"


def test_chain_depth_of_general_maps(tmp_path):
    """The longest merge chain bounds the passes a general map needs (host-only: handle creation)."""
    from blt_amd import synth
    L = _lib.lib()

    def depth(m):
        s = blt_amd.BpeStrategy(m)
        d = L.blt_debug_chain_depth(s.handle)
        s.close()
        return d
    assert depth({(97, 98): 256}) == 0                      # single-pass
    assert depth(synth.CHAINED_TEXT_MAP) == 2
    assert depth(synth.doubling_chain(24)) == 24
    assert depth({(97, 98): 65, (65, 99): 300, (300, 300): 301}) == 3
    assert depth(synth.SELF_VALUED_MAP) == 0                # "e " -> e: a value made from itself
    assert depth({(97, 98): 97}) == 0
    assert depth({(97, 98): 120, (120, 99): 97}) == 0      # a two-step cycle
    path = tmp_path / "wrap.txt"
    path.write_text(synth.wrap_merges_lines())
    s = blt_amd.BpeStrategy.from_file(str(path))
    assert L.blt_debug_chain_depth(s.handle) == 0           # (255, 255) -> 255


def test_workspace_size_of_cyclic_maps():
    """Host-only: a cyclic general map's workspace holds the sparse passes' bitmaps, lists and
    compaction words (about 1.75 n bytes more than a bounded map's), below 2^32 input bytes only."""
    from blt_amd import synth
    n, cs = 64 << 20, 1 << 20
    bounded = blt_amd.BpeStrategy(synth.CHAINED_TEXT_MAP)
    cyclic = blt_amd.BpeStrategy(synth.SELF_VALUED_MAP)
    single = blt_amd.BpeStrategy({(97, 98): 256})
    wb, wc, ws = (x.workspace_size(n, cs) for x in (bounded, cyclic, single))
    assert ws < wb < wc
    extra = wc - wb
    assert 1.70 * n < extra < 1.80 * n, extra / n
    big = 1 << 32   # positions past 32 bits: no sparse passes, no extra workspace
    assert cyclic.workspace_size(big, cs) == bounded.workspace_size(big, cs)
    for x in (bounded, cyclic, single):
        x.close()
