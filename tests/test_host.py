"""CPU: C-ABI library loads/exports, host BAM codec, header regeneration, synthetic generator."""
import ctypes
import hashlib
import struct

import numpy as np
import pytest

import bamutil
import oracle
from goldens import CASE_NAMES, GOLDEN, load_case
from openge_amd import lib as L


def test_library_exports_every_declared_symbol(built):
    so = ctypes.CDLL(str(L.LIB_PATH))
    missing = [s for s in L.exported_symbols() if not hasattr(so, s)]
    assert not missing, missing


def test_no_gpu_context_fails_loudly(built):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(L.OgeError, match="no HIP device"):
        L.Context(0)


@pytest.mark.parametrize("name", ["simple", "yhet208"])
def test_product_reader_matches_independent_parser(built, name):
    b = L.Bam(GOLDEN / "inputs" / load_case(name).meta["spec"]["file"])
    h, refs, recs, offs = bamutil.read_bam(GOLDEN / "inputs" / load_case(name).meta["spec"]["file"])
    assert b.n == len(offs) and b.n_ref == len(refs)
    assert np.array_equal(b.offs, offs)
    assert np.array_equal(b.recs[: len(recs)], recs)


def test_truncated_bgzf_is_an_error(built):
    with pytest.raises(L.OgeError, match="truncated"):
        L.Bam(GOLDEN / "inputs" / "208.truncated.bam")


def test_oversized_block_is_an_error(built, tmp_path):
    rec = bamutil.make_record("x", 0, 0, 10, "10M", "A" * 10)
    bad = struct.pack("<I", 10001) + rec[4:] + b"\0" * (10001 - len(rec) + 4)
    bamutil.write_bam_py(tmp_path / "bad.bam", "@HD\tVN:1.4\tSO:unsorted\n@SQ\tSN:c\tLN:100\n", [("c", 100)], [bad])
    with pytest.raises(L.OgeError, match="block size"):
        L.Bam(tmp_path / "bad.bam")


def _stream_digests(recs, offs):
    h, tail = hashlib.sha256(), []
    for o in offs:
        rb = bamutil.rec_bytes(recs, o)
        if int.from_bytes(rb[4:8], "little", signed=True) == -1:
            tail.append(rb)
        else:
            h.update(rb)
    return h.hexdigest(), hashlib.sha256(b"".join(sorted(tail))).hexdigest()


@pytest.mark.parametrize("name", CASE_NAMES)
def test_writer_reproduces_reference_output_stream(built, tmp_path, name):
    """Sorted order + 0x400 flags (from the oracle) written by the product BAM writer must give the
    reference's `mergesort -M` record stream byte for byte (bin recomputed, header regenerated)."""
    c = load_case(name)
    perm = oracle.sort_perm(c.recs, c.offs, c.n)
    so = c.offs[:-1][perm]
    dup, _ = oracle.markdup(c.recs, so, c.n, c.header)
    flags = np.array([int.from_bytes(c.recs[int(o) + 18:int(o) + 20].tobytes(), "little") for o in c.offs[:-1]],
                     dtype=np.uint16)
    d_in = np.empty(c.n, np.uint8)
    d_in[perm] = dup
    flags = np.where(d_in == 1, flags | 0x400, np.where(d_in == 0, flags & np.uint16(0xFBFF), flags)).astype(np.uint16)
    out = tmp_path / "o.bam"
    L.write_bam(out, c.header, c.recs, c.offs, c.n, order=perm.astype(np.uint32), flags=flags, sort_order=3)
    h, _, r, o = bamutil.read_bam(out)
    g = c.meta["sortdedup_v"]
    assert h == g["header"]
    ms, ts = _stream_digests(r, o)
    assert ms == g["mapped_sha256"] and ts == g["tail_multiset_sha256"]


def test_parallel_record_parse_equals_sequential(built, tmp_path):
    """bam_parse splits a >= 64 MB stream across threads (verified chain joins); the record offsets
    must equal the one-thread walk, also when a chunk boundary falls inside a record."""
    p = L.synth_params(160_000, preset="mix", seed=11)
    recs, offs, hdr = L.synth_host(p)
    path = tmp_path / "big.bam"
    L.write_bam(path, hdr, recs, offs, 320_000, level=1)
    one = L.Bam(path, threads=1)
    for t in (3, 8, 16):
        many = L.Bam(path, threads=t)
        assert many.n == one.n == 320_000
        assert np.array_equal(many.offs, one.offs)
        assert many.recs.tobytes() == one.recs.tobytes()


def test_synth_host_is_deterministic_and_thread_independent(built):
    p = L.synth_params(3000, preset="c2", seed=42)
    a, ao, _ = L.synth_host(p, threads=1)
    b, bo, _ = L.synth_host(L.synth_params(3000, preset="c2", seed=42), threads=7)
    assert np.array_equal(ao, bo) and np.array_equal(a, b)
    # records parse as BAM and every name appears exactly twice (one pair)
    names = [bamutil.fields(bamutil.rec_bytes(a, o))["name"] for o in ao[:-1]]
    from collections import Counter
    assert set(Counter(names).values()) == {2}


def test_synth_shape_c2(built):
    p = L.synth_params(20000, preset="c2", seed=1234)
    recs, offs, hdr = L.synth_host(p)
    n = 40000
    f = [bamutil.fields(bamutil.rec_bytes(recs, o)) for o in offs[:-1]]
    assert 280 <= offs[-1] / n <= 290                       # ~285 B/record
    assert sum(x["flag"] & 0x4 != 0 for x in f) / n == pytest.approx(0.0025, abs=0.002)
    assert len({x["refid"] for x in f}) == 24
    assert hdr.count("@RG") == 2


def test_bgzf_index_matches_framing(built, tmp_path):
    """oge_bgzf_index (host side of the GPU reader): deflate ranges, payload offsets and CRCs per
    block, empty blocks skipped, truncation and non-BGZF input rejected."""
    import zlib
    data = np.random.default_rng(7).integers(0, 4, 200_000, dtype=np.uint8).tobytes()
    blocks, want = [], []
    pos = zpos = 0
    for i in range(0, len(data), 65280):
        chunk = data[i:i + 65280]
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        body = c.compress(chunk) + c.flush()
        bsize = 18 + len(body) + 8
        blk = (b"\x1f\x8b\x08\x04\0\0\0\0\0\xff\x06\0BC\x02\0" + struct.pack("<H", bsize - 1) + body +
               struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk)))
        want.append((zpos + 18, zpos + bsize - 8, pos, zlib.crc32(chunk) & 0xFFFFFFFF))
        blocks.append(blk)
        pos += len(chunk)
        zpos += bsize
    eof = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    z = np.frombuffer(b"".join(blocks) + eof, dtype=np.uint8)
    lib = L.lib()
    nb = ctypes.c_uint64()
    assert lib.oge_bgzf_index(z.ctypes.data, len(z), None, None, None, None, 0, ctypes.byref(nb)) == -1  # cap 0: count only
    k = nb.value
    assert k == len(want)
    d0, d1, uo = (np.zeros(k + 1, dtype=np.uint64) for _ in range(3))
    crc = np.zeros(k, dtype=np.uint32)
    assert lib.oge_bgzf_index(z.ctypes.data, len(z), d0.ctypes.data, d1.ctypes.data, uo.ctypes.data, crc.ctypes.data, k,
                              ctypes.byref(nb)) == 0
    for i, (a, b, u, c) in enumerate(want):
        assert (d0[i], d1[i], uo[i], crc[i]) == (a, b, u, c)
    assert uo[k] == len(data)
    bad = z[:-100].copy()
    assert lib.oge_bgzf_index(bad.ctypes.data, len(bad), None, None, None, None, 0, ctypes.byref(nb)) != 0
    notgz = np.frombuffer(b"BAM\x01" + bytes(100), dtype=np.uint8)
    assert lib.oge_bgzf_index(notgz.ctypes.data, len(notgz), None, None, None, None, 0, ctypes.byref(nb)) != 0
