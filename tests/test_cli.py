"""The `blt` command line (blt_amd/csrc/blt_cli.cpp), a drop-in for the reference binary
(src/main.rs:8-60).  The GPU cases restate the reference's own CLI tests (tests/cli.rs:20-214)
and add chunked parity against the C oracle; the CPU cases cover argument handling, passthrough
(no tokenising) and the loud failure without a GPU.
"""
import os
import subprocess

import numpy as np
import pytest

from tests.conftest import ROOT

BLT = os.path.join(ROOT, "blt_amd", "blt")


def _gpu_present():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


def run(args, stdin=b"", **kw):
    if not os.path.exists(BLT):
        pytest.fail("blt_amd/blt is not built (run make)")
    return subprocess.run([BLT] + list(args), input=stdin, capture_output=True, timeout=300, **kw)


def basic(data: bytes) -> bytes:
    return bytes(np.frombuffer(data, np.uint8).astype(">u2").tobytes())


# ---- CPU: argument surface, passthrough, errors -------------------------------------------

def test_help_and_version():
    r = run(["--help"])
    assert r.returncode == 0
    for flag in ("--input", "--output", "--merges", "--passthrough", "--type", "--threads", "--memcap",
                 "--chunksize"):
        assert flag.encode() in r.stdout
    assert run(["-V"]).returncode == 0


def test_passthrough_mode():   # tests/cli.rs:195-214
    r = run(["--passthrough"], b"passthrough test")
    assert r.returncode == 0 and r.stdout == b"passthrough test"


def test_passthrough_with_type_prepends_token(tmp_path):   # lib.rs:284-293 runs for every strategy
    for name, tok in (("text", 0xFF01), ("audio", 0xFF02), ("bin", 0xFF03), ("video", 0xFF04)):
        r = run(["--passthrough", "--type", name], b"xy")
        assert r.returncode == 0 and r.stdout == bytes((tok >> 8, tok & 0xFF)) + b"xy"


def test_passthrough_files_and_large_stream(tmp_path):
    data = np.random.default_rng(5).integers(0, 256, 3 * (1 << 20) + 17, dtype=np.uint8).tobytes()
    src, dst = tmp_path / "in.bin", tmp_path / "out.bin"
    src.write_bytes(data)
    assert run(["--passthrough", "-i", str(src), "-o", str(dst), "--chunksize", "256KB"]).returncode == 0
    assert dst.read_bytes() == data
    r = run(["--passthrough", "--chunksize", "256KB", "--threads", "3"], data)
    assert r.returncode == 0 and r.stdout == data


def test_empty_input_writes_nothing(tmp_path):
    src = tmp_path / "empty"
    src.write_bytes(b"")
    r = run(["--passthrough", "-i", str(src)])
    assert r.returncode == 0 and r.stdout == b""


@pytest.mark.parametrize("args,msg", [
    (["--chunksize", "1GB"], b"Invalid unit or format: '1GB'"),
    (["--chunksize", "10.5MB"], b"Invalid number: '10.5'"),
    (["--merges", "/nonexistent/merges.txt"], b"Failed to load BPE merges"),
])
def test_config_errors_exit_1(args, msg):
    r = run(args + ["--passthrough"])
    assert r.returncode == 1
    assert msg in r.stderr


def test_invalid_merges_file_reports_line(tmp_path):
    m = tmp_path / "m.txt"
    m.write_text("97 98\nnot a pair\n")
    r = run(["--merges", str(m)], b"ab")
    assert r.returncode == 1 and b"Failed to load BPE merges" in r.stderr


@pytest.mark.parametrize("args", [["--bogus"], ["--type", "image"], ["--threads", "x"], ["--input"]])
def test_usage_errors_exit_2(args):
    r = run(args)
    assert r.returncode == 2 and b"error:" in r.stderr


def test_missing_input_file_fails(tmp_path):
    r = run(["-i", str(tmp_path / "nope"), "--passthrough"])
    assert r.returncode == 1


@pytest.mark.skipif(_gpu_present(), reason="checks the no-GPU failure")
def test_tokenising_without_gpu_fails_loudly():
    r = run([], b"hello")
    assert r.returncode == 1 and b"Error running tokenizer" in r.stderr and r.stdout == b""


# ---- GPU: the reference's CLI tests, then chunked parity ----------------------------------

@pytest.mark.gpu
def test_cli_stdin_stdout():   # tests/cli.rs:20-43
    r = run([], b"hello world")
    assert r.returncode == 0 and r.stdout == basic(b"hello world")


@pytest.mark.gpu
def test_cli_input_output_files(tmp_path):   # tests/cli.rs:45-80
    src, dst = tmp_path / "in.txt", tmp_path / "out.bin"
    src.write_bytes(b"hello from file")
    assert run(["--input", str(src), "--output", str(dst)]).returncode == 0
    assert dst.read_bytes() == basic(b"hello from file")


@pytest.mark.gpu
def test_cli_type_argument():   # tests/cli.rs:82-105
    r = run(["--type", "text"], b"test")
    assert r.returncode == 0 and r.stdout == b"\xff\x01" + basic(b"test")


@pytest.mark.gpu
def test_cli_bpe_merges(tmp_path):   # tests/cli.rs:107-140
    m = tmp_path / "merges.txt"
    m.write_bytes(b"97 98\n")
    r = run(["--merges", str(m)], b"ab c ab")
    exp = b"".join(int(t).to_bytes(2, "big") for t in (256, 32, 99, 32, 256))
    assert r.returncode == 0 and r.stdout == exp


@pytest.mark.gpu
@pytest.mark.parametrize("args,data", [(["--chunksize", "1KB"], b"some data"),   # tests/cli.rs:142-167
                                       (["--threads", "1"], b"thread test")])    # tests/cli.rs:169-193
def test_cli_chunksize_and_threads(args, data):
    r = run(args, data)
    assert r.returncode == 0 and r.stdout == basic(data)


def _merges_file(tmp_path, pairs):
    m = tmp_path / "merges.txt"
    m.write_text("".join(f"{a} {b}\n" for a, b in pairs))
    return m


@pytest.mark.gpu
@pytest.mark.parametrize("chunksize", ["256KB", "300000", "1MB"])
def test_cli_file_parity_many_chunks(tmp_path, chunksize):
    """mmap path: fixed chunks (pipeline.rs:73-81), window batching, --gpus; vs the C oracle."""
    from blt_amd import synth
    from oracle import oracle as O
    text = synth.text(5 * (1 << 20) + 4321, seed=11)
    pairs = synth.top_pair_merges(text, 300)
    m = _merges_file(tmp_path, pairs)
    merges = {(a, b): 256 + i for i, (a, b) in enumerate(pairs)}
    src, dst = tmp_path / "in.txt", tmp_path / "out.bin"
    src.write_bytes(text.tobytes())
    r = run(["--merges", str(m), "-i", str(src), "-o", str(dst), "--chunksize", chunksize, "--type", "bin"])
    assert r.returncode == 0, r.stderr
    cs = {"256KB": 256 << 10, "300000": 300000, "1MB": 1 << 20}[chunksize]
    exp = O.COracle(merges).run(text, cs, threads=4).tobytes()
    assert dst.read_bytes() == b"\xff\x03" + exp


@pytest.mark.gpu
def test_cli_stdin_regular_file_parity(tmp_path):
    """Stream path: from a regular file every read() returns a whole chunk, so the chunks are
    the fixed ones and the output equals the mmap path's."""
    from blt_amd import synth
    from oracle import oracle as O
    text = synth.text(3 * (1 << 20) + 99, seed=12)
    pairs = synth.top_pair_merges(text, 200)
    m = _merges_file(tmp_path, pairs)
    merges = {(a, b): 256 + i for i, (a, b) in enumerate(pairs)}
    src = tmp_path / "in.txt"
    src.write_bytes(text.tobytes())
    with open(src, "rb") as f:
        r = subprocess.run([BLT, "--merges", str(m), "--chunksize", "256KB", "--threads", "4"], stdin=f,
                           capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout == O.COracle(merges).run(text, 256 << 10, threads=4).tobytes()


@pytest.mark.gpu
def test_cli_basic_file_large(tmp_path):
    data = np.random.default_rng(3).integers(0, 256, (1 << 20) * 3 + 5, dtype=np.uint8).tobytes()
    src, dst = tmp_path / "in.bin", tmp_path / "out.bin"
    src.write_bytes(data)
    assert run(["-i", str(src), "-o", str(dst), "--chunksize", "256KB"]).returncode == 0
    assert dst.read_bytes() == basic(data)
