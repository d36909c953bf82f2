"""GPU: BGZF decompression (oge_bgzf_inflate[_dev]) and the device record-boundary walk
(oge_bam_record_offsets_dev).

Oracle: zlib.  Streams are made by zlib itself at levels 0 (stored), 1, 6, 9 and with the fixed-code
strategy, plus the GPU deflate's own output; the GPU must return exactly the bytes zlib compressed
(bit-exact), and must reject corrupt blocks (CRC or deflate errors) loudly.  The record walk must
equal the sequential block_size walk the reader does (bamio.cpp bam_parse)."""
import struct
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PAY = 65280


def bgzf(data: bytes, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, pay=PAY, eof=True) -> bytes:
    out = []
    for i in range(0, len(data), pay):
        chunk = data[i:i + pay]
        c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, strategy)
        body = c.compress(chunk) + c.flush()
        bsize = 18 + len(body) + 8
        out.append(b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" + struct.pack("<H", bsize - 1) + body +
                   struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk)))
    if eof:
        out.append(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))
    return b"".join(out)


def _bam_bytes(n_reads, seed=5):
    from openge_amd import lib as L
    p = L.synth_params(n_reads, preset="mix", seed=seed)
    recs, offs, _ = L.synth_host(p)
    return recs[: int(offs[-1])].tobytes()


DATA = {
    "bam": _bam_bytes(6_000),
    "text": (b"the quick brown fox jumps over the lazy dog; " * 9000)[:400_001],
    "random": np.random.default_rng(3).integers(0, 256, 150_000, dtype=np.uint8).tobytes(),
    "zeros": bytes(200_000),
    "one": b"Z",
    "acgt": bytes(np.random.default_rng(1).integers(0, 4, 300_000, dtype=np.uint8) + ord("A")),
}


@pytest.mark.parametrize("level", [0, 1, 6, 9])
@pytest.mark.parametrize("name", sorted(DATA))
def test_inflate_matches_zlib(ctx, name, level):
    data = DATA[name]
    assert ctx.bgzf_inflate(bgzf(data, level)) == data


@pytest.mark.parametrize("name", ["bam", "text", "acgt"])
def test_inflate_fixed_codes_and_rle(ctx, name):
    data = DATA[name]
    assert ctx.bgzf_inflate(bgzf(data, 6, zlib.Z_FIXED)) == data
    assert ctx.bgzf_inflate(bgzf(data, 6, zlib.Z_RLE)) == data
    assert ctx.bgzf_inflate(bgzf(data, 6, zlib.Z_HUFFMAN_ONLY)) == data


def _bgzf_ragged(data: bytes, sizes, level=6) -> bytes:
    out, i, k = [], 0, 0
    while i < len(data):
        n = sizes[k % len(sizes)]
        k += 1
        chunk = data[i:i + n]
        i += n
        c = zlib.compressobj(level, zlib.DEFLATED, -15)
        body = c.compress(chunk) + c.flush()
        out.append(b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" + struct.pack("<H", 18 + len(body) + 7) +
                   body + struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk)))
    return b"".join(out)


@pytest.mark.parametrize("level", [0, 6])
def test_inflate_ragged_payloads(ctx, level):
    """Payload sizes that leave every block at a different byte alignment (the lane decoder writes
    8-byte chunks and must not touch a neighbour's bytes), incl. 1-byte and 64 KiB payloads."""
    rng = np.random.default_rng(11)
    big = 65536 if level else 65280  # a stored 64 KiB payload does not fit a BGZF block
    sizes = [1, 7, big, 3, 65279, 12345] + rng.integers(1, big + 1, 40).tolist()
    data = DATA["bam"] + DATA["random"] + DATA["text"]
    assert ctx.bgzf_inflate(_bgzf_ragged(data, sizes, level)) == data


def _libdeflate():
    import ctypes as C
    try:
        ld = C.CDLL("libdeflate.so.0")
    except OSError:
        return None
    ld.libdeflate_alloc_compressor.restype = C.c_void_p
    ld.libdeflate_alloc_compressor.argtypes = [C.c_int]
    ld.libdeflate_deflate_compress.restype = C.c_size_t
    ld.libdeflate_deflate_compress.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.c_void_p, C.c_size_t]
    ld.libdeflate_free_compressor.argtypes = [C.c_void_p]
    return ld


@pytest.mark.parametrize("level", [1, 6, 9, 12])
def test_inflate_libdeflate_streams(ctx, level):
    """libdeflate (the host codec samtools-era writers use) emits one block per payload, with
    different Huffman shapes than zlib; level 12 gives near-optimal parses with long codes."""
    import ctypes as C
    ld = _libdeflate()
    if ld is None:
        pytest.skip("libdeflate.so.0 not loadable")
    comp = ld.libdeflate_alloc_compressor(level)
    data = DATA["bam"] + DATA["acgt"] + DATA["text"]
    out = []
    for i in range(0, len(data), PAY):
        chunk = data[i:i + PAY]
        buf = C.create_string_buffer(PAY + 1024)
        n = ld.libdeflate_deflate_compress(comp, chunk, len(chunk), buf, PAY + 1024)
        body = buf.raw[:n]
        out.append(b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" + struct.pack("<H", 18 + n + 7) + body +
                   struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk)))
    ld.libdeflate_free_compressor(comp)
    assert ctx.bgzf_inflate(b"".join(out)) == data


def test_inflate_full_64k_payloads(ctx):
    data = DATA["acgt"][:200_000]
    assert ctx.bgzf_inflate(bgzf(data, 6, pay=65536)) == data


def test_inflate_gpu_deflate_output(ctx):
    data = _bam_bytes(30_000, seed=8)
    z = ctx.bgzf_deflate(data, 6)
    assert ctx.bgzf_inflate(z) == data


def test_inflate_empty_and_eof_only(ctx):
    assert ctx.bgzf_inflate(b"") == b""
    assert ctx.bgzf_inflate(bgzf(b"")) == b""


def test_inflate_rejects_corruption(ctx):
    from openge_amd import lib as L
    z = bytearray(bgzf(DATA["bam"], 6))
    bad_crc = bytearray(z)
    bsize = struct.unpack_from("<H", z, 16)[0] + 1
    bad_crc[bsize - 8] ^= 0xFF  # first block's CRC
    with pytest.raises(L.OgeError, match="CRC"):
        ctx.bgzf_inflate(bytes(bad_crc))
    bad_body = bytearray(z)
    for k in range(40, 60):
        bad_body[k] ^= 0x5A
    with pytest.raises(L.OgeError):
        ctx.bgzf_inflate(bytes(bad_body))
    with pytest.raises(L.OgeError):
        ctx.bgzf_inflate(bytes(z[:-40]))  # truncated



@pytest.mark.parametrize("prep", ["0", "1"])
def test_inflate_header_prepass_on_and_off(ctx, monkeypatch, prep):
    """The header pre-pass (k_infl_prep: first deflate header of every BGZF block parsed and its tables
    built before phase 1) and phase 1's own in-loop header path (OGE_INFL_PREP=0, and whatever the pre-pass
    declines: stored first blocks, > 256 long codes, corrupt headers) give the same bytes and errors."""
    from openge_amd import lib as L
    monkeypatch.setenv("OGE_INFL_PREP", prep)
    for name in ("bam", "random", "text", "one"):
        for level in (0, 1, 6, 9):
            assert ctx.bgzf_inflate(bgzf(DATA[name], level)) == DATA[name]
        assert ctx.bgzf_inflate(bgzf(DATA[name], 6, zlib.Z_FIXED)) == DATA[name]
    z = bytearray(bgzf(DATA["bam"], 6))
    z[18] ^= 0x06  # the first block's BTYPE bits: dynamic -> fixed (decodes garbage: an error)
    with pytest.raises(L.OgeError):
        ctx.bgzf_inflate(bytes(z))
    z = bytearray(bgzf(DATA["bam"], 6))
    for k in range(21, 40):  # inside the first header's code-length data
        z[k] ^= 0xA5
    with pytest.raises(L.OgeError):
        ctx.bgzf_inflate(bytes(z))


def test_inflate_carry_over_on_one_context(ctx):
    """One context, calls in sequence: a corrupt stream (phase 1 fails some blocks, so phase 2 may not clear
    every bitmap word it would), then a valid stream, then a smaller one, then a larger one -- each checked
    byte for byte.  The phase-1 bitmap buffer is carried from call to call as known-clear."""
    from openge_amd import lib as L
    big = DATA["bam"] + DATA["text"] + DATA["random"]
    z = bytearray(bgzf(big, 6))
    for k in range(200, 240):  # the first block's body: a deflate error, not only a CRC one
        z[k] ^= 0x5A
    with pytest.raises(L.OgeError):
        ctx.bgzf_inflate(bytes(z))
    for data in (big, DATA["acgt"], DATA["bam"][:70_001], big + DATA["zeros"]):
        assert ctx.bgzf_inflate(bgzf(data, 6)) == data
    assert ctx.bgzf_inflate(bgzf(DATA["text"], 6, zlib.Z_FIXED)) == DATA["text"]


def _stream(n_pairs, seed):
    """A decompressed BAM stream (header + records) and its record offsets, from the host writer."""
    from openge_amd import lib as L
    p = L.synth_params(n_pairs, preset="mix", seed=seed)
    recs, offs, hdr = L.synth_host(p)
    import tempfile, os, gzip
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "x.bam")
        L.write_bam(path, hdr, recs, offs, len(offs) - 1, level=1)
        raw = gzip.decompress(open(path, "rb").read())
    l_text = struct.unpack_from("<I", raw, 4)[0]
    q = 8 + l_text
    n_ref = struct.unpack_from("<I", raw, q)[0]
    q += 4
    for _ in range(n_ref):
        ln = struct.unpack_from("<I", raw, q)[0]
        q += 4 + ln + 4
    want = [q]
    while want[-1] < len(raw):
        want.append(want[-1] + 4 + struct.unpack_from("<I", raw, want[-1])[0])
    assert want[-1] == len(raw)
    return raw, q, n_ref, np.array(want, dtype=np.uint64)


@pytest.mark.parametrize("n_pairs,seed", [(1, 1), (300, 2), (60_000, 3)])
def test_record_offsets_equal_sequential_walk(ctx, n_pairs, seed):
    import torch
    raw, base, n_ref, want = _stream(n_pairs, seed)
    dev = torch.device("cuda", 0)
    d = torch.frombuffer(bytearray(raw + bytes(64)), dtype=torch.uint8).to(dev)
    torch.cuda.synchronize()
    n = ctx.record_offsets_dev(d.data_ptr(), base, len(raw), n_ref)
    assert n == len(want) - 1
    off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ctx.record_offsets_dev(d.data_ptr(), base, len(raw), n_ref, off.data_ptr(), n + 1)
    torch.cuda.synchronize()
    assert np.array_equal(off.cpu().numpy().view(np.uint64), want)


def test_record_offsets_reject_bad_block_size(ctx):
    import torch
    from openge_amd import lib as L
    raw, base, n_ref, want = _stream(40_000, 4)
    bad = bytearray(raw)
    k = int(want[len(want) // 2])
    struct.pack_into("<I", bad, k, 20000)  # block_size > 10000 (bam_deserializer.h:160-163)
    dev = torch.device("cuda", 0)
    d = torch.frombuffer(bytearray(bytes(bad) + bytes(64)), dtype=torch.uint8).to(dev)
    torch.cuda.synchronize()
    with pytest.raises(L.OgeError):
        ctx.record_offsets_dev(d.data_ptr(), base, len(bad), n_ref)


@pytest.mark.parametrize("level", [1, 6, 9])
def test_inflate_host_writer_streams(ctx, tmp_path, level):
    """BGZF written by the host writer (libdeflate when present, else zlib) -- the CLI's own inputs."""
    import gzip
    from openge_amd import lib as L
    # 240k reads (~68 MB, ~1000 blocks): enough back-references just beyond the decoder's LDS ring
    # (the case a flush race once corrupted)
    p = L.synth_params(120_000, preset="c2", seed=31)
    recs, offs, hdr = L.synth_host(p, threads=8)
    path = tmp_path / "w.bam"
    L.write_bam(str(path), hdr, recs, offs, len(offs) - 1, level=level)
    z = path.read_bytes()
    assert ctx.bgzf_inflate(z) == gzip.decompress(z)


def test_long_codes_before_direct_literal_runs(ctx):
    """Dynamic-Huffman blocks with explicit code lengths (tests/deflate_craft.py): 15-bit literal codes
    mixed at random with 6-bit ones, so a long code followed by three direct-table (<= 6-bit) literals
    starts a decode step at every fill level of the lane decoder's bit buffer, including a buffer
    refilled to exactly 32 bits.  A literal batch after a long code needs 15 + 3 * 6 = 33 bits (VERDICT
    r02: commit 3941758 allowed it and corrupted a block at 300M reads; only the CRC caught it); the
    decode must be exact and the always-on bit-budget guard silent."""
    import deflate_craft as D
    for seed in (7, 8):
        data, z = D.long_short_stream(130, seed=seed)  # two waves' worth of blocks
        assert ctx.bgzf_inflate(z) == data
