"""Test-side RFC 1951 reader and a CPU restatement of the GPU deflate's Huffman length builder.

`parse_block(raw)` walks one raw deflate stream (pure Python, table driven) and returns, per deflate
block, its type, the code lengths its header transmits (literal/length, distance, code-length code)
and the symbol counts its body actually uses -- enough to check an encoder's header against the
frequencies it encoded.

`huff_lengths(f, M)` restates `huff_lengths` of openge_amd/csrc/bgzf.hip (the k_defl_huff kernel):
two-queue Huffman over the used symbols ranked by (frequency, symbol), depths clamped to M, the
per-depth counts repaired to an exactly complete code (lengthen the longest code < M while
over-subscribed, shorten the longest code that fits while under-subscribed), lengths handed out
longest-first to the least frequent symbols.  `header_lengths(counts)` restates the whole header
construction of k_defl_huff: EOB counted once, at least two codes per tree, the lengths run-length
coded (RFC 1951 3.2.7, the kernel's run rules) and the code-length code built with M = 7.
Our own deflate has no reference counterpart (OpenGE calls zlib, util/bgzf_output_stream.cpp:74-79),
so these pin the GPU encoder to its documented algorithm, not to zlib's bytes.
"""
from __future__ import annotations

KLIT, KDIST, KCL = 286, 30, 19
CL_ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258]
LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DEXT = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]


class _Bits:
    def __init__(self, b: bytes):
        self.b = bytes(b) + b"\0" * 8
        self.p = 0

    def peek(self) -> int:  # >= 25 bits from the current position
        q = self.p >> 3
        return int.from_bytes(self.b[q:q + 4], "little") >> (self.p & 7)

    def get(self, n: int) -> int:
        v = self.peek() & ((1 << n) - 1) if n else 0
        self.p += n
        return v


def _table(lens: list[int]) -> list:
    """15-bit direct table over LSB-first bit strings: entry = (symbol, length) or None."""
    mx = max(lens) if lens else 0
    bl = [0] * 16
    for L in lens:
        if L:
            bl[L] += 1
    code, nxt = 0, [0] * 16
    for b in range(1, 16):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    t = [None] * (1 << 15)
    for s, L in enumerate(lens):
        if not L:
            continue
        c = nxt[L]
        nxt[L] += 1
        r = int(format(c, f"0{L}b")[::-1], 2)
        for k in range(1 << (15 - L)):
            t[r | (k << L)] = (s, L)
    assert mx <= 15
    return t


def _dec(bits: _Bits, t: list) -> int:
    e = t[bits.peek() & 0x7FFF]
    if e is None:
        raise ValueError("invalid code")
    bits.p += e[1]
    return e[0]


def parse_block(raw: bytes) -> list[dict]:
    """Deflate blocks of one raw deflate stream: [{type, lit, dist, cl, lit_count, dist_count, out}]."""
    bits = _Bits(raw)
    blocks, out = [], bytearray()
    while True:
        fin, typ = bits.get(1), bits.get(2)
        d = {"type": typ}
        if typ == 0:
            bits.p = (bits.p + 7) & ~7
            n, nn = bits.get(16), bits.get(16)
            assert n ^ 0xFFFF == nn
            q = bits.p >> 3
            out += bits.b[q:q + n]
            bits.p += 8 * n
        else:
            if typ == 1:
                lit = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
                dist = [5] * 30
                cl = None
            else:
                assert typ == 2
                hlit, hdist, hclen = bits.get(5) + 257, bits.get(5) + 1, bits.get(4) + 4
                cl = [0] * KCL
                for i in range(hclen):
                    cl[CL_ORDER[i]] = bits.get(3)
                ct = _table(cl)
                lens: list[int] = []
                while len(lens) < hlit + hdist:
                    s = _dec(bits, ct)
                    if s < 16:
                        lens.append(s)
                    elif s == 16:
                        lens += [lens[-1]] * (3 + bits.get(2))
                    elif s == 17:
                        lens += [0] * (3 + bits.get(3))
                    else:
                        lens += [0] * (11 + bits.get(7))
                lit, dist = lens[:hlit], lens[hlit:]
            lt, dt = _table(lit), _table(dist)
            lc, dc = [0] * 288, [0] * 30
            while True:
                s = _dec(bits, lt)
                lc[s] += 1
                if s < 256:
                    out.append(s)
                elif s == 256:
                    break
                else:
                    c = s - 257
                    ln = LBASE[c] + bits.get(LEXT[c])
                    ds = _dec(bits, dt)
                    dc[ds] += 1
                    dd = ds + 1 if ds < 4 else ((2 + (ds & 1)) << ((ds - 2) >> 1)) + 1 + bits.get(DEXT[ds])
                    for _ in range(ln):
                        out.append(out[-dd])
            d.update(lit=lit, dist=dist, cl=cl, lit_count=lc, dist_count=dc)
        blocks.append(d)
        if fin:
            break
    blocks[-1]["out"] = bytes(out)
    return blocks


# ---------------------------------------------------------------------------------------- builder
def huff_lengths(f: list[int], M: int) -> list[int]:
    """bgzf.hip huff_lengths, restated."""
    n = len(f)
    order = sorted((i for i in range(n) if f[i]), key=lambda i: (f[i], i))
    m = len(order)
    lens = [0] * n
    if m == 0:
        return lens
    if m == 1:
        lens[order[0]] = 1
        return lens
    w = [f[i] for i in order] + [0] * (m - 1)
    parent = [0] * (2 * m - 1)
    i, j, nx = 0, m, m
    for _ in range(m - 1):
        pick = []
        for _ in range(2):
            if i < m and (j >= nx or w[i] <= w[j]):
                pick.append(i)
                i += 1
            else:
                pick.append(j)
                j += 1
        a, b = pick
        w[nx] = w[a] + w[b]
        parent[a] = parent[b] = nx
        nx += 1
    root = 2 * m - 2
    depth = [0] * (2 * m - 1)
    for x in range(root - 1, -1, -1):  # parents have larger indices
        depth[x] = depth[parent[x]] + 1
    cnt = [0] * (M + 1)
    for k in range(m):
        cnt[min(depth[k], M)] += 1
    one = 1 << M
    K = sum(cnt[b] << (M - b) for b in range(1, M + 1))
    while K > one:
        b = M - 1
        while cnt[b] == 0:
            b -= 1
        cnt[b] -= 1
        cnt[b + 1] += 1
        K -= 1 << (M - b - 1)
    while K < one:
        b = M
        while cnt[b] == 0 or K + (1 << (M - b)) > one:
            b -= 1
        cnt[b] -= 1
        cnt[b - 1] += 1
        K += 1 << (M - b)
    k = 0
    for b in range(M, 0, -1):
        for _ in range(cnt[b]):
            lens[order[k]] = b
            k += 1
    return lens


def _at_least_two(f: list[int]) -> list[int]:
    f = list(f)
    nz = sum(1 for x in f if x)
    i = 0
    while nz < 2 and i < len(f):
        if not f[i]:
            f[i] = 1
            nz += 1
        i += 1
    return f


def header_lengths(lit_count: list[int], dist_count: list[int]) -> tuple[list[int], list[int], list[int]]:
    """k_defl_huff's transmitted lengths for a block whose body uses these symbol counts:
    (literal/length lengths [hlit], distance lengths [hdist], code-length-code lengths [19])."""
    f = list(lit_count[:KLIT]) + [0] * max(0, KLIT - len(lit_count))
    f[256] = 1
    f = _at_least_two(f)
    fd = _at_least_two(list(dist_count[:KDIST]))
    ll, dl = huff_lengths(f, 15), huff_lengths(fd, 15)
    a = KLIT
    while a > 257 and ll[a - 1] == 0:
        a -= 1
    b = KDIST
    while b > 1 and dl[b - 1] == 0:
        b -= 1
    fcl = [0] * KCL
    for seq in (ll[:a], dl[:b]):
        i, N = 0, len(seq)
        while i < N:
            v, run = seq[i], 1
            while i + run < N and seq[i + run] == v:
                run += 1
            if v == 0 and run >= 3:
                r = min(run, 138)
                fcl[18 if r >= 11 else 17] += 1
                i += r
                continue
            fcl[v] += 1
            i += 1
            rest = run - 1
            if v != 0:
                while rest >= 3:
                    r = min(rest, 6)
                    fcl[16] += 1
                    rest -= r
                    i += r
    cl = huff_lengths(_at_least_two(fcl), 7)
    return ll[:a], dl[:b], cl
