"""Test-side raw DEFLATE writer with EXPLICIT Huffman code lengths (RFC 1951 3.2.2 / 3.2.7), pure Python.

zlib chooses its own code lengths from symbol frequencies; the inflate tests also need streams whose
codes have chosen lengths -- e.g. many 15-bit literal codes next to many 6-bit ones, so that a long
code is followed by runs of short ones at every bit-buffer fill level of the lane decoder
(inflate_lane.hip).  Only literals and the end-of-block code are emitted (no matches), with every
code-length-code length 4 (a complete code over the 16 plain lengths, no run-length symbols)."""
from __future__ import annotations

import struct
import zlib

import numpy as np


class BitWriter:
    def __init__(self):
        self.acc = 0
        self.n = 0
        self.out = bytearray()

    def put(self, v: int, nb: int) -> None:  # LSB first
        self.acc |= (v & ((1 << nb) - 1)) << self.n
        self.n += nb
        while self.n >= 8:
            self.out.append(self.acc & 0xFF)
            self.acc >>= 8
            self.n -= 8

    def bytes(self) -> bytes:
        if self.n:
            self.out.append(self.acc & 0xFF)
            self.acc, self.n = 0, 0
        return bytes(self.out)


def canonical_codes(lengths) -> list[int]:
    """Canonical codes (RFC 1951 3.2.2), already bit-reversed for LSB-first emission."""
    mx = max(lengths) if len(lengths) else 0
    bl = [0] * (mx + 2)
    for L in lengths:
        if L:
            bl[L] += 1
    code, nxt = 0, [0] * (mx + 2)
    for b in range(1, mx + 1):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    out = []
    for L in lengths:
        if L:
            c = nxt[L]
            nxt[L] += 1
            out.append(int(format(c, f"0{L}b")[::-1], 2))
        else:
            out.append(0)
    return out


def kraft(lengths) -> float:
    return sum(2.0 ** -L for L in lengths if L)


def dynamic_literal_block(data: bytes, lit_lengths: list[int], final: bool = True) -> bytes:
    """One dynamic-Huffman block holding `data` as literals, with the given literal/length code lengths
    (index 0..285; 256 = end of block must be non-zero); two 1-bit distance codes (unused)."""
    assert len(lit_lengths) == 286 and lit_lengths[256]
    assert abs(kraft(lit_lengths) - 1.0) < 1e-12, "literal/length code must be complete"
    for b in set(data):
        assert lit_lengths[b], f"byte {b} has no code"
    dist_lengths = [1, 1]
    lit_codes = canonical_codes(lit_lengths)
    w = BitWriter()
    w.put(1 if final else 0, 1)
    w.put(2, 2)  # dynamic
    hlit = 286
    while hlit > 257 and lit_lengths[hlit - 1] == 0:
        hlit -= 1
    w.put(hlit - 257, 5)
    w.put(len(dist_lengths) - 1, 5)
    w.put(19 - 4, 4)  # HCLEN: all 19 code-length-code lengths
    order = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
    cl_len = [4 if s < 16 else 0 for s in range(19)]
    for s in order:
        w.put(cl_len[s], 3)
    cl_codes = canonical_codes(cl_len)
    for L in lit_lengths[:hlit] + dist_lengths:
        w.put(cl_codes[L], 4)
    for b in data:
        w.put(lit_codes[b], lit_lengths[b])
    w.put(lit_codes[256], lit_lengths[256])
    return w.bytes()


def bgzf_member(payload: bytes, body: bytes) -> bytes:
    bsize = 18 + len(body) + 8
    assert bsize <= 65536
    return (b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" + struct.pack("<H", bsize - 1) + body +
            struct.pack("<II", zlib.crc32(payload) & 0xFFFFFFFF, len(payload)))


def long_short_lengths(rng: np.random.Generator, n6: int = 60, n15: int = 128) -> tuple[list[int], list[int], list[int]]:
    """Literal/length lengths with n6 6-bit literals, n15 15-bit codes (one of them end-of-block), and
    7-/8-bit codes completing the Kraft sum.  -> (lengths, short literals, long literals)."""
    units = 32768 - n6 * 512 - n15  # in 2^-15
    assert units >= 0
    n7, rest = divmod(units, 256)
    n8, rest = divmod(rest, 128)
    n9, rest = divmod(rest, 64)
    n10, rest = divmod(rest, 32)
    n11, rest = divmod(rest, 16)
    n12, rest = divmod(rest, 8)
    n13, rest = divmod(rest, 4)
    n14, rest = divmod(rest, 2)
    extra15 = rest
    lens_needed = [6] * n6 + [7] * n7 + [8] * n8 + [9] * n9 + [10] * n10 + [11] * n11 + [12] * n12 + [13] * n13 + \
        [14] * n14 + [15] * (n15 + extra15 - 1)
    assert len(lens_needed) <= 256, "too many codes for the literal alphabet"
    syms = rng.permutation(256)[:len(lens_needed)]
    L = [0] * 286
    for s, ln in zip(syms, lens_needed):
        L[int(s)] = ln
    L[256] = 15
    short = [int(s) for s, ln in zip(syms, lens_needed) if ln == 6]
    long = [int(s) for s, ln in zip(syms, lens_needed) if ln == 15]
    assert abs(kraft(L) - 1.0) < 1e-12
    return L, short, long


def long_short_stream(n_blocks: int, seed: int = 7) -> tuple[bytes, bytes]:
    """BGZF blocks whose payloads mix 15-bit and 6-bit literal codes at random (p_long 0.25..0.55):
    a 15-bit code followed by three 6-bit codes falls at every bit-buffer fill level many times per
    block.  -> (payload bytes concatenated, BGZF stream with EOF block)."""
    rng = np.random.default_rng(seed)
    data, z = [], []
    for k in range(n_blocks):
        L, short, long = long_short_lengths(rng, n6=int(rng.integers(48, 62)), n15=int(rng.integers(64, 129)))
        p_long = 0.25 + 0.30 * rng.random()
        n = int(rng.integers(20_000, 36_000)) + k  # ragged sizes
        pick_long = rng.random(n) < p_long
        vals = np.where(pick_long, rng.choice(long, n), rng.choice(short, n)).astype(np.uint8)
        payload = vals.tobytes()
        data.append(payload)
        z.append(bgzf_member(payload, dynamic_literal_block(payload, L)))
    z.append(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))
    return b"".join(data), b"".join(z)
