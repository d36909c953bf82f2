"""CPU: the test-side deflate reader (tests/deflate_parse.py) against zlib, and the restated Huffman length
builder of the GPU deflate (bgzf.hip huff_lengths) on its own properties: complete codes (Kraft sum 1), the
length limit, monotone in frequency, and plain Huffman lengths wherever no depth exceeds the limit."""
import heapq
import zlib

import numpy as np
import pytest

import deflate_parse as DP


@pytest.mark.parametrize("level,kind", [(1, "text"), (6, "c2like"), (9, "random"), (0, "random"), (6, "runs")])
def test_reader_matches_zlib(level, kind):
    rng = np.random.default_rng(level)
    if kind == "text":
        data = b"the quick brown fox jumps over the lazy dog " * 800
    elif kind == "random":
        data = rng.integers(0, 256, 30000, dtype=np.uint8).tobytes()
    elif kind == "runs":
        data = bytes(np.repeat(rng.integers(0, 4, 3000, dtype=np.uint8), rng.integers(1, 40, 3000)))[:60000]
    else:
        data = (rng.integers(33, 75, 40000, dtype=np.uint8).tobytes() + b"frag0000123" * 500)
    co = zlib.compressobj(level, zlib.DEFLATED, -15)
    z = co.compress(data) + co.flush()
    blocks = DP.parse_block(z)
    assert blocks[-1]["out"] == data
    for b in blocks:
        if b["type"] == 2:  # every used symbol has a code
            assert all(b["lit"][s] for s, c in enumerate(b["lit_count"][:len(b["lit"])]) if c)


def _plain_huffman_depths(f):
    h = [(w, i, (i,)) for i, w in enumerate(f) if w]
    heapq.heapify(h)
    d = [0] * len(f)
    k = len(f)
    while len(h) > 1:
        wa, ia, la = heapq.heappop(h)
        wb, ib, lb = heapq.heappop(h)
        for s in la + lb:
            d[s] += 1
        heapq.heappush(h, (wa + wb, k, la + lb))
        k += 1
    return d


@pytest.mark.parametrize("seed", range(6))
def test_restated_builder_properties(seed):
    rng = np.random.default_rng(seed)
    for n, M in ((286, 15), (30, 15), (19, 7)):
        for shape in ("uniform", "geometric", "fib"):
            if shape == "uniform":
                f = rng.integers(0, 1000, n).tolist()
            elif shape == "geometric":
                f = [int(1e6 * 0.6 ** (i % 40)) + (i % 3) for i in rng.permutation(n)]
            else:
                a, b, fib = 1, 1, []
                for _ in range(n):
                    fib.append(a)
                    a, b = b, min(a + b, 1 << 40)
                f = [fib[i] for i in rng.permutation(n)]
            L = DP.huff_lengths(f, M)
            used = [i for i in range(n) if f[i]]
            assert all(L[i] for i in used) and all(not L[i] for i in range(n) if not f[i])
            assert max(L) <= M
            if len(used) >= 2:
                assert sum(2.0 ** -L[i] for i in used) == 1.0
            for i in used:  # a more frequent symbol never gets a longer code
                for j in used:
                    if f[i] > f[j]:
                        assert L[i] <= L[j]
            d = _plain_huffman_depths(f)
            if len(used) >= 2 and max(d) <= M:  # no clamp: optimal total cost
                assert sum(f[i] * L[i] for i in used) == sum(f[i] * d[i] for i in used)
