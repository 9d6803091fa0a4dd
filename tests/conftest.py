import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")


@pytest.fixture(scope="session")
def kats():
    with open(os.path.join(GOLDEN, "reference_kats.json")) as f:
        return json.load(f)


def merges_dict(triples):
    """[[a, b, v], ...] -> {(a, b): v}; a later duplicate overwrites (HashMap collect)."""
    d = {}
    for a, b, v in triples:
        d[(a, b)] = v
    return d


def tokens_be(tokens):
    out = bytearray()
    for t in tokens:
        out += bytes(((t >> 8) & 0xFF, t & 0xFF))
    return bytes(out)
