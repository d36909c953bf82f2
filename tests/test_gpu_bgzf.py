"""GPU: BGZF compression on the device (oge_bgzf_deflate[_dev]) and the device-side writer helpers.

Compressed bytes are not part of parity; the checks are the size-independent
properties of the format: every block is a valid gzip member with the BGZF `BC` extra field and a
BSIZE that matches, zlib inflates it back to exactly the input slice (65,280-byte payloads), CRC-32
and ISIZE agree, the output is deterministic, and level 0 gives stored blocks."""
import struct
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PAY = 65280


def split_blocks(z: bytes):
    """Parse a BGZF stream into (payload, deflate_bytes) per block, checking the framing."""
    out, p = [], 0
    while p < len(z):
        assert z[p:p + 4] == b"\x1f\x8b\x08\x04", f"bad magic at {p}"
        xlen = struct.unpack_from("<H", z, p + 10)[0]
        assert xlen == 6 and z[p + 12:p + 14] == b"BC" and struct.unpack_from("<H", z, p + 14)[0] == 2
        bsize = struct.unpack_from("<H", z, p + 16)[0] + 1
        assert p + bsize <= len(z)
        body = z[p + 18:p + bsize - 8]
        crc, isize = struct.unpack_from("<II", z, p + bsize - 8)
        d = zlib.decompressobj(-15)
        payload = d.decompress(body)
        assert d.eof and not d.unused_data, f"block at {p}: trailing bytes in the deflate stream"
        assert len(payload) == isize
        assert zlib.crc32(payload) & 0xFFFFFFFF == crc
        out.append((payload, body))
        p += bsize
    return out


def check_roundtrip(data: bytes, z: bytes):
    blocks = split_blocks(z)
    assert len(blocks) == (len(data) + PAY - 1) // PAY
    assert b"".join(b[0] for b in blocks) == data
    for i, (payload, _) in enumerate(blocks):
        assert len(payload) == min(PAY, len(data) - i * PAY)
    return blocks


def _bam_bytes(n_reads, seed=5):
    from openge_amd import lib as L
    p = L.synth_params(n_reads, preset="mix", seed=seed)
    recs, offs, _ = L.synth_host(p)
    return recs[: int(offs[-1])].tobytes()


CASES = {
    "one_byte": b"A",
    "short_text": b"the quick brown fox jumps over the lazy dog " * 3,
    "exact_block": bytes(np.random.default_rng(1).integers(0, 4, PAY, dtype=np.uint8) + ord("A")),
    "block_plus_one": bytes(np.random.default_rng(2).integers(0, 4, PAY + 1, dtype=np.uint8) + ord("A")),
    "zeros": bytes(300_000),
    "random": np.random.default_rng(3).integers(0, 256, 200_000, dtype=np.uint8).tobytes(),
    "runs": b"".join(bytes([c]) * int(k) for c, k in zip(np.random.default_rng(4).integers(0, 256, 3000),
                                                             np.random.default_rng(5).integers(1, 300, 3000))),
}


@pytest.mark.parametrize("level", [6, 8, 9])
@pytest.mark.parametrize("name", sorted(CASES))
def test_deflate_roundtrip(ctx, name, level):
    data = CASES[name]
    z = ctx.bgzf_deflate(data, level)
    check_roundtrip(data, z)


def test_deflate_chain_levels(ctx):
    """Levels 8 / 9 walk same-prefix chains with lazy matching: valid BGZF, deterministic, and no larger
    than level 6 on BAM records (zlib-6 printed beside them)."""
    data = _bam_bytes(40_000, seed=9)
    sizes = {}
    for level in (6, 8, 9):
        z = ctx.bgzf_deflate(data, level)
        assert z == ctx.bgzf_deflate(data, level)
        check_roundtrip(data, z)
        sizes[level] = len(z)
    ref = sum(len(zlib.compress(data[i:i + PAY], 6)) for i in range(0, len(data), PAY))
    print(f"\nBAM payload {len(data)} B: level 6 {sizes[6]}, 8 {sizes[8]}, 9 {sizes[9]}; zlib-6 {ref}")
    assert sizes[8] <= sizes[6] and sizes[9] <= sizes[6]


def test_deflate_empty(ctx):
    assert ctx.bgzf_deflate(b"", 6) == b""


def test_deflate_bam_records_ratio_and_determinism(ctx):
    data = _bam_bytes(40_000)
    z1 = ctx.bgzf_deflate(data, 6)
    z2 = ctx.bgzf_deflate(data, 6)
    assert z1 == z2
    blocks = check_roundtrip(data, z1)
    ref = sum(len(zlib.compress(data[i:i + PAY], 6)) for i in range(0, len(data), PAY))
    ratio = len(z1) / len(data)
    n_stored = sum(1 for p, b in blocks if b[0] == 1 and len(b) == len(p) + 5)
    print(f"\nBAM payload {len(data)} B -> GPU {len(z1)} B ({ratio:.3f}); zlib-6 per block {ref} B "
          f"({ref / len(data):.3f}); stored blocks {n_stored}")
    assert len(z1) < 1.15 * ref + 26 * len(blocks)


def test_level0_is_stored(ctx):
    data = _bam_bytes(2_000)
    z = ctx.bgzf_deflate(data, 0)
    for payload, body in check_roundtrip(data, z):
        assert body[0] == 1 and len(body) == len(payload) + 5


def test_incompressible_falls_back_to_stored(ctx):
    data = CASES["random"]
    z = ctx.bgzf_deflate(data, 6)
    for payload, body in check_roundtrip(data, z):
        assert len(body) <= len(payload) + 5


@pytest.mark.parametrize("shift", [0, 1, 2, 3, 5])
def test_deflate_dev_unaligned_source(ctx, shift):
    import torch
    from openge_amd import lib as L
    data = _bam_bytes(3_000, seed=9)[: 3 * PAY + 777]
    dev = torch.device("cuda", 0)
    buf = torch.zeros(len(data) + 64, dtype=torch.uint8, device=dev)
    buf[shift:shift + len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    cap = int(L.lib().oge_bgzf_bound(len(data)))
    dst = torch.empty(cap, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    got = ctx.bgzf_deflate_dev(buf.data_ptr() + shift, len(data), 6, dst.data_ptr(), cap)
    torch.cuda.synchronize()
    check_roundtrip(data, dst[:got].cpu().numpy().tobytes())


def test_deflate_dev_rejects_small_capacity(ctx):
    import torch
    from openge_amd import lib as L
    dev = torch.device("cuda", 0)
    src = torch.zeros(1000, dtype=torch.uint8, device=dev)
    dst = torch.empty(100, dtype=torch.uint8, device=dev)
    with pytest.raises(L.OgeError):
        ctx.bgzf_deflate_dev(src.data_ptr(), 1000, 6, dst.data_ptr(), 100)


def test_fix_bins_and_drop_flagged(ctx):
    import torch
    from openge_amd import lib as L
    p = L.synth_params(20_000, preset="mix", seed=21)
    recs, offs, _ = L.synth_host(p)
    n = len(offs) - 1
    recs = recs.copy()
    o = offs[:-1].astype(np.int64)
    bins = recs[o + 14].astype(np.uint16) | (recs[o + 15].astype(np.uint16) << 8)
    rng = np.random.default_rng(0)
    dup = rng.random(n) < 0.2
    recs[o[dup] + 19] |= 0x04  # FLAG 0x400
    broken = recs.copy()
    broken[o + 14] = 0x5A
    broken[o + 15] = 0xA5
    dev = torch.device("cuda", 0)
    d_r = torch.from_numpy(broken).to(dev)
    d_o = torch.from_numpy(offs.view(np.int64)).to(dev)
    torch.cuda.synchronize()
    ctx.fix_bins_dev(d_r.data_ptr(), d_o.data_ptr(), n)
    torch.cuda.synchronize()
    fixed = d_r.cpu().numpy()
    assert np.array_equal(fixed[o + 14].astype(np.uint16) | (fixed[o + 15].astype(np.uint16) << 8), bins)
    d_out = torch.empty_like(d_r)
    d_oo = torch.empty_like(d_o)
    m = ctx.drop_flagged_dev(d_r.data_ptr(), d_o.data_ptr(), n, 0x400, d_out.data_ptr(), d_oo.data_ptr())
    torch.cuda.synchronize()
    assert m == int((~dup).sum())
    oo = d_oo.cpu().numpy().view(np.uint64)[: m + 1]
    got = d_out.cpu().numpy()[: int(oo[m])].tobytes()
    keep = np.nonzero(~dup)[0]
    want = b"".join(recs[offs[i]:offs[i + 1]].tobytes() for i in keep)
    assert got == want


def _fib_bytes(n, seed):
    """bytes whose frequencies follow the Fibonacci numbers (22 symbols): plain Huffman depths reach ~21,
    so the 15-bit limit, the clamp and the Kraft repair of the GPU's length builder all run"""
    f, a, b = [], 1, 1
    for _ in range(22):
        f.append(a)
        a, b = b, a + b
    sym = np.repeat(np.arange(22, dtype=np.uint8) * 7 + 3, f)
    rng = np.random.default_rng(seed)
    return bytes(rng.permutation(np.resize(sym, n)))


HUFF_CASES = {
    "c2_records": lambda: _bam_bytes(6_000),
    "fibonacci": lambda: _fib_bytes(3 * PAY, 1),
    "geometric": lambda: bytes(np.minimum(np.random.default_rng(7).geometric(0.18, 2 * PAY), 255).astype(np.uint8)),
    "runs": lambda: CASES["runs"],
    "short_text": lambda: CASES["short_text"],
}


@pytest.mark.parametrize("name", sorted(HUFF_CASES))
def test_deflate_header_equals_restated_builder(ctx, name):
    """every dynamic block's transmitted code lengths (literal/length, distance and
    code-length code) equal the CPU restatement of k_defl_huff (tests/deflate_parse.py) applied to the
    symbol counts the block's body uses -- the length-limited two-queue Huffman with Kraft repair pinned
    independently of round trips."""
    import deflate_parse as DP
    data = HUFF_CASES[name]()
    z = ctx.bgzf_deflate(data, 6)
    n_dyn = 0
    for payload, body in check_roundtrip(data, z):
        blocks = DP.parse_block(body)
        assert blocks[-1]["out"] == payload
        for b in blocks:
            if b["type"] != 2:
                continue
            n_dyn += 1
            lit, dist, cl = DP.header_lengths(b["lit_count"], b["dist_count"])
            assert b["lit"] == lit and b["dist"] == dist and b["cl"] == cl
    assert n_dyn > 0


def test_deflate_bytes_pinned(ctx):
    """The GPU deflate's exact output bytes on a fixed input (the C2 generator, 20,000 pairs, seed 99 --
    the c2_20k golden set -- as one record stream, level 6) against a committed sha256
    (tests/golden/deflate_sha.json, written by tools/deflate_sha.py on the GPU box): "same bytes" claims
    about deflate changes are this test."""
    import hashlib
    import json
    from pathlib import Path
    from openge_amd import lib as L
    p = L.synth_params(20_000, preset="c2", seed=99)
    recs, offs, _ = L.synth_host(p)
    data = recs[:int(offs[-1])].tobytes()
    z = ctx.bgzf_deflate(data, 6)
    want = json.loads((Path(__file__).parent / "golden" / "deflate_sha.json").read_text())
    assert len(data) == want["input_bytes"]
    assert len(z) == want["output_bytes"] and hashlib.sha256(z).hexdigest() == want["sha256"]
