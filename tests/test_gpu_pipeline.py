"""GPU: the device BGZF framing index and the whole `mergesort [-M]` chain on a BAM file resident in
HBM (oge_mergesort_bgzf_dev), against the host framing walk and the REFERENCE's own outputs
(tests/golden, made by oracle/_ref from the reference's modules; MergeSortCommand::runCommand,
commands/command_mergesort.cpp:68-117)."""
import gzip
import hashlib
import struct
import zlib

import numpy as np
import pytest
import torch

import bamutil
from goldens import CASE_NAMES, GOLDEN, load_case
from openge_amd import lib as L
from test_gpu_cli import case_input, digests

pytestmark = pytest.mark.gpu


def _host_index(z: bytes):
    import ctypes as C
    a = np.frombuffer(z, np.uint8)
    nb = C.c_uint64()
    L.lib().oge_bgzf_index(a.ctypes.data, len(a), None, None, None, None, 0, C.byref(nb))
    n = nb.value
    ix = np.zeros(3 * n + 1, np.uint64)
    crc = np.zeros(max(n, 1), np.uint32)
    L.check(L.lib().oge_bgzf_index(a.ctypes.data, len(a), ix.ctypes.data, ix[n:].ctypes.data, ix[2 * n:].ctypes.data,
                                   crc.ctypes.data, n, C.byref(nb)))
    return n, ix, crc[:n]


def _dev_index(ctx, z: bytes):
    dz = torch.from_numpy(np.frombuffer(z + b"\0" * 8, np.uint8).copy()).cuda()
    n = ctx.bgzf_index_dev(dz.data_ptr(), len(z))
    ix = torch.zeros(3 * n + 1, dtype=torch.int64, device="cuda")
    crc = torch.zeros(max(n, 1), dtype=torch.int32, device="cuda")
    p = ix.data_ptr()
    n2 = ctx.bgzf_index_dev(dz.data_ptr(), len(z), p, p + 8 * n, p + 16 * n, crc.data_ptr(), n)
    assert n2 == n
    ctx.sync()
    return n, ix.cpu().numpy().view(np.uint64), crc.cpu().numpy().view(np.uint32)[:n]


def _streams():
    p = L.synth_params(20_000, preset="c2", seed=5)
    recs, offs, hdr = L.synth_host(p)
    raw = recs[:int(offs[-1])].tobytes()
    yield "zlib6", bamutil.bgzf_blocks(raw, 6)
    yield "zlib0", bamutil.bgzf_blocks(raw[:300_000], 0)
    # empty blocks in the middle and a gzip member whose extra field holds a second subfield
    co = zlib.compressobj(6, zlib.DEFLATED, -15)
    c = co.compress(b"") + co.flush()
    empty = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, ord("B"), ord("C"), 2, 18 + len(c) + 8 - 1) + c + \
        struct.pack("<II", 0, 0)
    chunk = raw[:5000]
    co = zlib.compressobj(6, zlib.DEFLATED, -15)
    d = co.compress(chunk) + co.flush()
    xf = b"XY" + struct.pack("<H", 3) + b"abc" + b"BC" + struct.pack("<HH", 2, 18 + 7 + len(d) + 8 - 1)
    two = struct.pack("<BBBBIBBH", 31, 139, 8, 4, 0, 0, 255, len(xf)) + xf + d + \
        struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk))
    yield "empty+xfield", empty + bamutil.bgzf_blocks(raw[:200_000], 6)[:-28] + empty + two + empty
    # a fake block header planted inside a stored block's payload: the candidate chain is not exact,
    # the host walk decides
    fake = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, ord("B"), ord("C"), 2, 40) + b"\0" * 30
    yield "planted", bamutil.bgzf_blocks(raw[:70_000] + fake + raw[70_000:150_000], 0)
    # hundreds of tiny blocks: more candidates per 4096-byte scan block than the counting pass stashes
    # (kStash), so the second scan places them; and runs of them next to ordinary blocks
    tiny = b"".join(bamutil.bgzf_blocks(raw[i:i + 3], 6)[:-28] for i in range(0, 3000, 3))
    yield "tiny_blocks", tiny + bamutil.bgzf_blocks(raw[:100_000], 6)
    for name in ("simple.bam", "208.yhet.bam"):
        yield name, (GOLDEN / "inputs" / name).read_bytes()


def _planted_chains():
    """A level-0 stream of several MiB with a false three-header chain planted inside a stored payload just
    past every 1 MiB segment boundary of the device index's segment walk: each segment's guess is the false
    chain, whose walk breaks, and the join re-walks the segment from its predecessor's exit."""
    p = L.synth_params(10_000, preset="c2", seed=9)
    recs, offs, hdr = L.synth_host(p)
    z = bytearray(bamutil.bgzf_blocks(recs[:int(offs[-1])].tobytes(), 0))
    n, hix, _ = _host_index(bytes(z))
    starts = sorted(int(x) - 18 for x in hix[:n])  # d0 = start + 12 + xlen (6): the block starts
    fake = b"".join(struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, ord("B"), ord("C"), 2, 39) + b"\0" * 22
                    for _ in range(3))
    planted = 0
    for k in range(1, len(z) >> 20):
        q = (k << 20) + 64
        nxt = min(x for x in starts if x >= (k << 20))
        prv = max(x for x in starts if x < (k << 20))
        if prv + 18 + 5 <= q and q + len(fake) + 8 < nxt:
            z[q:q + len(fake)] = fake
            planted += 1
    assert planted >= 3 and len(z) > 4 << 20
    return bytes(z)


@pytest.mark.parametrize("mode", ["segments", "scan"])
@pytest.mark.parametrize("name,z", list(_streams()) + [("planted_chains", _planted_chains())],
                         ids=lambda x: x if isinstance(x, str) else "")
def test_device_bgzf_index_equals_host_walk(ctx, name, z, mode, monkeypatch):
    """The segment walk (r06 default) and the byte scan it falls back to (OGE_BGZF_INDEX=scan) both equal the
    host walk; the scan hands planted false headers to the host walk, the segment walk walks past them."""
    if mode == "scan":
        monkeypatch.setenv("OGE_BGZF_INDEX", "scan")
    n, hix, hcrc = _host_index(z)
    m, dix, dcrc = _dev_index(ctx, z)
    assert m == n
    assert np.array_equal(dix[:3 * n + 1], hix) and np.array_equal(dcrc, hcrc)


def test_device_bgzf_index_errors_like_host(ctx):
    z = (GOLDEN / "inputs" / "208.truncated.bam").read_bytes()
    with pytest.raises(L.OgeError, match="truncated"):
        _dev_index(ctx, z)


def _run_pipeline(ctx, src_bytes: bytes, **kw):
    dz = torch.from_numpy(np.frombuffer(src_bytes + b"\0" * 8, np.uint8).copy()).cuda()
    o = L.mergesort_opts(**kw)
    d, nb, nr, nd = ctx.mergesort_bgzf_dev(dz.data_ptr(), len(src_bytes), o)
    out = np.empty(nb, np.uint8)
    L.check(L.lib().oge_memcpy(ctx.h, out.ctypes.data, d, nb, 2), ctx.h)
    return out.tobytes(), nr, nd


@pytest.fixture(scope="module", params=CASE_NAMES)
def case(request, built):
    return load_case(request.param)


def test_pipeline_mergesort_M_matches_reference(ctx, case, tmp_path):
    src = case_input(case, tmp_path).read_bytes()
    out, nr, nd = _run_pipeline(ctx, src, mark_duplicates=1)
    (tmp_path / "o.bam").write_bytes(out)
    h, m, t = digests(tmp_path / "o.bam")
    g = case.meta["sortdedup_v"]
    assert h == g["header"] and m == g["mapped_sha256"] and t == g["tail_multiset_sha256"]
    assert nr == case.n
    assert out[-28:] == bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def test_pipeline_sort_and_remove_match_reference(ctx, case, tmp_path):
    src = case_input(case, tmp_path).read_bytes()
    out, nr, _ = _run_pipeline(ctx, src)
    (tmp_path / "s.bam").write_bytes(out)
    h, m, t = digests(tmp_path / "s.bam")
    assert h == case.meta["sorted_header"] and m == case.meta["sort"]["mapped_sha256"]
    out, nr, _ = _run_pipeline(ctx, src, mark_duplicates=1, remove_duplicates=1)
    (tmp_path / "r.bam").write_bytes(out)
    _, _, recs, offs = bamutil.read_bam(tmp_path / "r.bam")
    assert nr == len(offs) == case.n - case.meta["sortdedup_v"]["n_dup"]
    assert not (bamutil.flags_of(recs, offs) & 0x400).any()


def test_pipeline_program_line_and_levels(ctx, tmp_path):
    src = (GOLDEN / "inputs" / "208.yhet.bam").read_bytes()
    ref = None
    for level in (0, 1, 6, 9):
        out, _, _ = _run_pipeline(ctx, src, mark_duplicates=1, level=level, program_line=b"openge mergesort -M x")
        raw = gzip.decompress(out)
        if ref is None:
            ref = raw
        assert raw == ref
    (tmp_path / "p.bam").write_bytes(out)
    h = bamutil.read_bam(tmp_path / "p.bam")[0]
    pg = [l for l in h.splitlines() if l.startswith("@PG")]
    assert pg[-1] == "@PG\tID:openge\tCL:openge mergesort -M x\tVN:0.3-dev"  # after the input's own @PG lines


@pytest.mark.parametrize("slots", ["1", "8", "300"])
def test_record_walk_slots(ctx, monkeypatch, tmp_path, slots):
    """The record walk's fill expands the count walk's per-chunk record slots; a chunk with more records
    than slots (OGE_RECWALK_SLOTS forces it) is walked again.  Same output either way, with the slots in
    their own workspace (a fresh context: the sorted-records arena is not there yet) and in that arena."""
    p = L.synth_params(60_000, preset="mix", seed=17)
    recs, offs, hdr = L.synth_host(p)
    L.write_bam(tmp_path / "in.bam", hdr, recs, offs, len(offs) - 1, level=1)
    src = (tmp_path / "in.bam").read_bytes()
    want = _run_pipeline(ctx, src, mark_duplicates=1)
    monkeypatch.setenv("OGE_RECWALK_SLOTS", slots)
    fresh = L.Context(0)
    try:
        assert _run_pipeline(fresh, src, mark_duplicates=1) == want
        assert _run_pipeline(fresh, src, mark_duplicates=1) == want
    finally:
        fresh.close()


def _run_host_pipeline(ctx, src_bytes: bytes, **kw):
    hz = torch.from_numpy(np.frombuffer(src_bytes, np.uint8).copy()).pin_memory()
    cap = len(src_bytes) * 2 + (1 << 20)
    ho = torch.empty(cap, dtype=torch.uint8).pin_memory()
    o = L.mergesort_opts(**kw)
    nb, nr, nd = ctx.mergesort_bgzf_host(hz.data_ptr(), len(src_bytes), o, ho.data_ptr(), cap)
    return ho[:nb].numpy().tobytes(), nr, nd


@pytest.mark.parametrize("groups,seg,direct", [("8", "32768", "1"), ("8", "32768", "0"), ("7", "3", "0"), ("1", "1", "0"),
                                               ("64", "2", "1")])
def test_host_pipeline_equals_device_chain(ctx, monkeypatch, tmp_path, groups, seg, direct):
    """oge_mergesort_bgzf_host (file in host memory, chunked upload, host framing index; the deflate
    straight into the page-locked output, or segments copied down while the next is compressed) writes the
    same bytes as the chain on a resident file."""
    monkeypatch.setenv("OGE_HOSTPIPE_GROUPS", groups)
    monkeypatch.setenv("OGE_HOSTPIPE_SEG_BLOCKS", seg)
    monkeypatch.setenv("OGE_HOSTPIPE_DIRECT", direct)
    p = L.synth_params(60_000, preset="c2", seed=11)
    recs, offs, hdr = L.synth_host(p)
    L.write_bam(tmp_path / "in.bam", hdr, recs, offs, len(offs) - 1, level=6)
    src = (tmp_path / "in.bam").read_bytes()
    for kw in ({"mark_duplicates": 1}, {}, {"mark_duplicates": 1, "remove_duplicates": 1, "level": 1}):
        want = _run_pipeline(ctx, src, **kw)
        got = _run_host_pipeline(ctx, src, **kw)
        assert got[1:] == want[1:] and got[0] == want[0], kw


@pytest.mark.parametrize("name", ["208.yhet.bam", "simple.bam"])
def test_host_pipeline_reference_inputs(ctx, monkeypatch, name):
    monkeypatch.setenv("OGE_HOSTPIPE_GROUPS", "5")
    monkeypatch.setenv("OGE_HOSTPIPE_SEG_BLOCKS", "1")
    src = (GOLDEN / "inputs" / name).read_bytes()
    assert _run_host_pipeline(ctx, src, mark_duplicates=1) == _run_pipeline(ctx, src, mark_duplicates=1)


def test_host_pipeline_errors(ctx):
    z = (GOLDEN / "inputs" / "208.truncated.bam").read_bytes()
    with pytest.raises(L.OgeError, match="truncated"):
        _run_host_pipeline(ctx, z, mark_duplicates=1)
    src = (GOLDEN / "inputs" / "208.yhet.bam").read_bytes()
    hz = np.frombuffer(src, np.uint8).copy()
    ho = np.empty(64, np.uint8)
    with pytest.raises(L.OgeError, match="too small"):
        ctx.mergesort_bgzf_host(hz.ctypes.data, len(src), L.mergesort_opts(), ho.ctypes.data, len(ho))


def test_host_pipeline_failed_segment_drains(ctx, monkeypatch, tmp_path):
    """A segment that fails after earlier segments' device-to-host copies were queued: the call returns its
    error only once those copies (and the uploads) are done, so the page-locked buffers can be reused or
    freed at once; the next call on the same buffers and context writes the right bytes."""
    monkeypatch.setenv("OGE_HOSTPIPE_GROUPS", "7")
    monkeypatch.setenv("OGE_HOSTPIPE_SEG_BLOCKS", "2")
    p = L.synth_params(30_000, preset="c2", seed=5)
    recs, offs, hdr = L.synth_host(p)
    L.write_bam(tmp_path / "in.bam", hdr, recs, offs, len(offs) - 1, level=6)
    src = (tmp_path / "in.bam").read_bytes()
    want = _run_pipeline(ctx, src, mark_duplicates=1)
    hz = torch.from_numpy(np.frombuffer(src, np.uint8).copy()).pin_memory()
    cap = len(src) * 2 + (1 << 20)
    ho = torch.zeros(cap, dtype=torch.uint8).pin_memory()
    o = L.mergesort_opts(mark_duplicates=1)
    monkeypatch.setenv("OGE_HOSTPIPE_FAIL_SEG", "3")
    with pytest.raises(L.OgeError, match="injected segment failure"):
        ctx.mergesort_bgzf_host(hz.data_ptr(), len(src), o, ho.data_ptr(), cap)
    before = ho.clone()  # whatever the queued copies wrote is complete now: nothing may change any more
    torch.cuda.synchronize()
    assert torch.equal(before, ho)
    ho.fill_(0)
    monkeypatch.delenv("OGE_HOSTPIPE_FAIL_SEG")
    nb, nr, nd = ctx.mergesort_bgzf_host(hz.data_ptr(), len(src), o, ho.data_ptr(), cap)
    assert (ho[:nb].numpy().tobytes(), nr, nd) == want
