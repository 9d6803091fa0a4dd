"""Committed golden fixtures (tests/golden/fixtures.json, made by tests/golden/make_fixtures.py
from the KAT-pinned oracle): the oracle must still reproduce them on CPU, and the GPU library
through the C ABI on a GPU."""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _cases():
    with open(os.path.join(HERE, "golden", "fixtures.json")) as f:
        return json.load(f)["cases"]


def _merges(c):
    return {(a, b): v for a, b, v in c["merges"]} if c["merges"] or c["name"] == "empty" else None


@pytest.mark.parametrize("case", _cases(), ids=lambda c: c["name"])
def test_oracle_reproduces_fixture(case):
    from oracle import oracle as O
    data = bytes.fromhex(case["input_hex"])
    out = O.run_chunks(data, case["chunk_size"], merges=_merges(case), passthrough=case["passthrough"],
                       content_type=case["content_type"])
    assert out.hex() == case["output_hex"]
    if _merges(case) is not None and not case["passthrough"]:
        c = O.COracle(_merges(case)).run(np.frombuffer(data, np.uint8), case["chunk_size"],
                                         content_type=case["content_type"], threads=2)
        assert bytes(c).hex() == case["output_hex"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", _cases(), ids=lambda c: c["name"])
def test_gpu_reproduces_fixture(case):
    import blt_amd
    data = bytes.fromhex(case["input_hex"])
    strategy = blt_amd.select_strategy(_merges(case), passthrough=case["passthrough"])
    out = blt_amd.run_tokenizer(data, case["chunk_size"], strategy, content_type=case["content_type"])
    assert out.hex() == case["output_hex"]
