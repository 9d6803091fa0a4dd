"""Generates tests/golden/fixtures.json: small input/output vectors of the BPE path.

    python tests/golden/make_fixtures.py

The outputs come from the CPU restatement (oracle/), which tests/test_oracle_kats.py pins to
every known-answer test of the reference (reference_kats.json).  The reference itself cannot
run here (Rust toolchain absent), so these vectors extend the pinned oracle to inputs the
reference's tests do not cover: chunk ends, content-type tokens, multi-pass maps, the basic
strategy.  Regenerate only when the oracle changes; the tests compare both the oracle and the
GPU library against the committed file.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle as O  # noqa: E402


def seeded_bytes(seed, n, alphabet):
    return np.random.default_rng(seed).integers(0, alphabet, n, dtype=np.uint8).tobytes()


def main():
    cases = []

    def add(name, data, merges, chunk_size, content_type=None, passthrough=False):
        out = O.run_chunks(data, chunk_size, merges=merges, passthrough=passthrough, content_type=content_type)
        cases.append({
            "name": name,
            "input_hex": data.hex(),
            "merges": [[a, b, v] for (a, b), v in sorted((merges or {}).items())],
            "chunk_size": chunk_size,
            "content_type": content_type,
            "passthrough": passthrough,
            "output_hex": bytes(out).hex(),
        })

    text = b"the quick brown fox jumps over the lazy dog and the other dog. " * 9
    m_text = {(116, 104): 256, (104, 101): 257, (256, 101): 258, (32, 116): 259, (111, 103): 260, (100, 111): 261}
    add("text_small_map_one_chunk", text, m_text, 1 << 20)
    add("text_small_map_chunk_97", text, m_text, 97, content_type="text")
    dense = {(a, b): 256 + 8 * a + b for a in range(8) for b in range(8) if (a ^ b) & 1}
    add("random8_dense_map_chunk_100", seeded_bytes(7, 1000, 8), dense, 100, content_type="bin")
    add("random8_dense_map_chunk_1", seeded_bytes(8, 64, 8), dense, 1)
    chained = {(97, 97): 97}                                   # tokenizer.rs:204-212 style
    add("chained_aa_to_a", b"a" * 77 + b"b" + b"a" * 5, chained, 1 << 20)
    bytev = {(101, 32): 256, (256, 116): 257, (116, 104): 65, (65, 101): 258}  # byte-valued merge
    add("byte_valued_chain", b"the the then thee e t " * 7, bytev, 33, content_type="audio")
    add("basic_random", seeded_bytes(9, 300, 256), None, 128)
    add("passthrough", seeded_bytes(10, 50, 256), None, 16, passthrough=True)
    add("empty", b"", m_text, 16)
    with open(os.path.join(HERE, "fixtures.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_fixtures.py", "oracle": "oracle/oracle.py run_chunks",
                   "cases": cases}, f, indent=1)
    print(f"{len(cases)} fixtures")


if __name__ == "__main__":
    main()
