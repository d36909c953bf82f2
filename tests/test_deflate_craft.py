"""CPU: the explicit-code-length DEFLATE writer of tests/deflate_craft.py produces valid streams (zlib
inflates them to their payloads) with the code-length mix the GPU inflate test needs: many 15-bit
literal codes beside 6-bit ones."""
import gzip

import numpy as np

import deflate_craft as D


def test_crafted_streams_inflate_with_zlib():
    data, z = D.long_short_stream(12, seed=3)
    assert gzip.decompress(z) == data


def test_crafted_code_lengths_are_complete_and_mixed():
    rng = np.random.default_rng(1)
    for _ in range(20):
        L, short, long = D.long_short_lengths(rng, n6=int(rng.integers(48, 62)), n15=int(rng.integers(64, 129)))
        assert abs(D.kraft(L) - 1.0) < 1e-12
        assert len(short) >= 48 and len(long) >= 60
        assert all(L[s] == 6 for s in short) and all(L[s] == 15 for s in long)
