"""The Python binding surface: ByteTokenizer / load_bpe_merges / version / __version__.

Restates the reference binding's own tests (blt_python/tests/test_tokenizer.py:14-45 construction
and validation, :131-156 BPE, :222-270 utilities and module attributes) against blt_amd, and adds
bit-exact checks of tokenize_file's output files (the reference tests only check that output
exists).  CPU cases need no GPU (construction, validation, empty input, the loader); GPU cases run
the library's file pipeline (blt_run_tokenizer) and compare with the C oracle.
"""
import os

import numpy as np
import pytest

import blt_amd as blt
from blt_amd import BltError


def _basic(data: bytes) -> bytes:
    return np.frombuffer(data, np.uint8).astype(">u2").tobytes()


# ---- construction and validation (test_tokenizer.py:14-45) -------------------------------

def test_basic_tokenizer_creation():
    t = blt.ByteTokenizer()
    assert t is not None
    assert "ByteTokenizer" in str(t)
    assert repr(t) == "ByteTokenizer(merges=0, content_type=None, threads=None, chunk_size=None, memory_cap=None)"


def test_tokenizer_with_merges():
    t = blt.ByteTokenizer(merges={(97, 98): 256, (99, 100): 257})
    assert "merges=2" in str(t)


def test_tokenizer_with_content_type():
    assert 'content_type=Some("Text")' in str(blt.ByteTokenizer(content_type="Text"))
    assert 'content_type=Some("Bin")' in str(blt.ByteTokenizer(content_type="Bin"))


def test_repr_of_every_option():   # lib.rs:162-170, Rust {:?} of each Option
    t = blt.ByteTokenizer(merges={(1, 2): 300}, content_type="Bin", threads=2, chunk_size="1MB", memory_cap=50)
    assert repr(t) == ('ByteTokenizer(merges=1, content_type=Some("Bin"), threads=Some(2), '
                       'chunk_size=Some("1MB"), memory_cap=Some(50))')


@pytest.mark.parametrize("ct", ["Invalid", "text", "Audio", "Video", ""])
def test_invalid_content_type(ct):   # only "Text" / "Bin" (lib.rs:66-75)
    with pytest.raises(ValueError):
        blt.ByteTokenizer(content_type=ct)


def test_invalid_memory_cap():
    with pytest.raises(ValueError):
        blt.ByteTokenizer(memory_cap=150)   # over 100 %
    blt.ByteTokenizer(memory_cap=100)
    blt.ByteTokenizer(memory_cap=0)
    # u8 extraction (PyO3): out of range is an OverflowError, not a ValueError
    with pytest.raises(OverflowError):
        blt.ByteTokenizer(memory_cap=256)
    with pytest.raises(OverflowError):
        blt.ByteTokenizer(memory_cap=-1)


def test_merges_types_are_checked():   # HashMap<(u8, u8), u16> extraction
    with pytest.raises(OverflowError):
        blt.ByteTokenizer(merges={(256, 1): 300})
    with pytest.raises(OverflowError):
        blt.ByteTokenizer(merges={(1, 2): 70000})
    with pytest.raises(TypeError):
        blt.ByteTokenizer(merges={(1, 2): "x"})


# ---- utilities and module attributes (test_tokenizer.py:222-270) ---------------------------

def test_version_function():
    v = blt.version()
    assert isinstance(v, str) and len(v) > 0 and "." in v


def test_module_version_and_exports():
    assert blt.__version__ == blt.version()
    for name in ("ByteTokenizer", "load_bpe_merges", "version", "__version__"):
        assert hasattr(blt, name), name


def test_load_bpe_merges_file_not_found():
    with pytest.raises(IOError):
        blt.load_bpe_merges("non_existent_file.txt")


def test_load_bpe_merges_valid_file(tmp_path):
    p = tmp_path / "m.txt"
    p.write_text("97 98\n99 100\n")
    m = blt.load_bpe_merges(str(p))
    assert isinstance(m, dict) and len(m) == 2
    assert m[(97, 98)] == 256 and m[(99, 100)] == 257


# ---- tokenize_file --------------------------------------------------------------------------

def test_empty_input(tmp_path):   # test_tokenizer.py:70-93: no chunks, so no GPU is touched
    src, dst = tmp_path / "in", tmp_path / "out"
    src.write_bytes(b"")
    blt.ByteTokenizer().tokenize_file(str(src), str(dst))
    assert dst.exists() and dst.read_bytes() == b""


def test_empty_input_with_content_type(tmp_path):   # the token is written before any chunk
    src, dst = tmp_path / "in", tmp_path / "out"
    src.write_bytes(b"")
    blt.ByteTokenizer(content_type="Bin").tokenize_file(str(src), str(dst))
    assert dst.read_bytes() == b"\xff\x03"


def test_missing_input_raises_not_found(tmp_path):   # File::open in setup_io (io_handler.rs:57)
    with pytest.raises(BltError) as e:
        blt.ByteTokenizer().tokenize_file(str(tmp_path / "nope"), str(tmp_path / "out"))
    assert e.value.kind == "NotFound" and "os error 2" in str(e.value)
    assert not (tmp_path / "out").exists()   # the output is created only after the input opened


def test_bad_chunk_size_raises(tmp_path):
    src = tmp_path / "in"
    src.write_bytes(b"x")
    with pytest.raises(BltError) as e:
        blt.ByteTokenizer(chunk_size="1GB").tokenize_file(str(src), str(tmp_path / "out"))
    assert "Invalid unit or format" in str(e.value)


@pytest.mark.gpu
def test_basic_tokenization(tmp_path):   # test_tokenizer.py:47-68, with the exact bytes
    src, dst = tmp_path / "in", tmp_path / "out"
    src.write_bytes(b"hello world")
    blt.ByteTokenizer().tokenize_file(str(src), str(dst))
    assert dst.read_bytes() == _basic(b"hello world")


@pytest.mark.gpu
def test_bpe_tokenization(tmp_path):   # test_tokenizer.py:131-156
    src, dst = tmp_path / "in", tmp_path / "out"
    src.write_bytes(b"ab")
    blt.ByteTokenizer(merges={(97, 98): 256}).tokenize_file(str(src), str(dst))
    assert dst.read_bytes() == b"\x01\x00"


@pytest.mark.gpu
def test_configuration_options_and_content_type(tmp_path):   # test_tokenizer.py:181-205
    src, dst = tmp_path / "in", tmp_path / "out"
    src.write_bytes(b"test data for configuration")
    blt.ByteTokenizer(threads=2, chunk_size="1MB", memory_cap=50, content_type="Text").tokenize_file(str(src), str(dst))
    assert dst.read_bytes() == b"\xff\x01" + _basic(b"test data for configuration")


def test_dict_ids_follow_the_loader():
    """lib.rs:103-114 writes the keys to a merges file and loads it: ids 256 + key order, values
    ignored.  A dict whose values chain (120 feeds (120, 99)) is then single-pass; with
    use_dict_ids its values are the ids and it is not.  No GPU: handle creation is host-only."""
    merges = {(97, 98): 120, (120, 99): 300, (100, 100): 97}
    s = blt.ByteTokenizer(merges=merges)._strategy()
    assert s.info() == (3, True)
    s.close()
    s = blt.ByteTokenizer(merges=merges, use_dict_ids=True)._strategy()
    assert s.info() == (3, False)
    s.close()


def test_dict_ids_wrap_like_the_loader():
    """Every byte pair as a key: the loader's u16 counter wraps after 65,280 lines
    (config_loader.rs:18, :40), so the last 256 keys get ids 0..255 and the map needs passes."""
    merges = {(a, b): 1 for a in range(256) for b in range(256)}
    s = blt.ByteTokenizer(merges=merges)._strategy()
    assert s.info() == (65536, False)
    s.close()


@pytest.mark.gpu
def test_large_data_bpe_bit_exact(tmp_path):
    """A multi-chunk file with a 300-pair merge map: ids 256 + the dict's key order (the
    reference binding's temporary merges file), then with use_dict_ids the dict's values; both
    against the C oracle chunked at the same size."""
    from blt_amd import synth
    from oracle import oracle as O
    text = synth.text(3 * (1 << 20) + 12345, seed=21)
    pairs = synth.top_pair_merges(text, 300)
    rng = np.random.default_rng(4)
    ids = rng.permutation(np.arange(256, 256 + 300))
    merges = {p: int(i) for p, i in zip(pairs, ids)}
    src, dst = tmp_path / "in", tmp_path / "out"
    src.write_bytes(text.tobytes())
    blt.ByteTokenizer(merges=merges, chunk_size="256KB", content_type="Bin").tokenize_file(str(src), str(dst))
    line_ids = {p: 256 + i for i, p in enumerate(merges)}
    exp = O.COracle(line_ids).run(text, 256 << 10, threads=4).tobytes()
    assert dst.read_bytes() == b"\xff\x03" + exp
    blt.ByteTokenizer(merges=merges, chunk_size="256KB", content_type="Bin",
                      use_dict_ids=True).tokenize_file(str(src), str(dst))
    exp = O.COracle(merges).run(text, 256 << 10, threads=4).tobytes()
    assert dst.read_bytes() == b"\xff\x03" + exp


@pytest.mark.gpu
def test_chained_merges_from_dict(tmp_path):
    """With use_dict_ids, a dict whose values feed other keys needs several passes
    (tokenizer.rs:63-86)."""
    from oracle import oracle as O
    merges = {(97, 98): 120, (120, 99): 300, (100, 100): 97}
    data = (b"abcabcddbxabc" * 5000)
    src, dst = tmp_path / "in", tmp_path / "out"
    src.write_bytes(data)
    blt.ByteTokenizer(merges=merges, chunk_size="256KB", use_dict_ids=True).tokenize_file(str(src), str(dst))
    exp = O.COracle(merges).run(np.frombuffer(data, np.uint8), 256 << 10, threads=2).tobytes()
    assert dst.read_bytes() == exp


@pytest.mark.gpu
def test_performance_benchmark(tmp_path):   # test_tokenizer.py:272-306: 100 KiB in under 1 s
    import time
    src, dst = tmp_path / "in", tmp_path / "out"
    src.write_bytes(b"x" * (100 * 1024))
    t0 = time.time()
    blt.ByteTokenizer().tokenize_file(str(src), str(dst))
    assert time.time() - t0 < 1.0
    assert dst.read_bytes() == _basic(b"x" * (100 * 1024))
