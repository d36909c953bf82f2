"""GPU: ONE BGZF BAM file decoded by G ranks from their own byte ranges (oge_bgzf_decode_shard /
oge_mergesort_bgzf_shard, openge_amd/csrc/shard.hip) -- config 4's input path: every rank inflates only
the blocks that start in its range, the ranks join their block and record boundaries, the record that
straddles a part's end is handed to the rank it starts in.  The reference reads the file on one thread
(util/bgzf_input_stream.cpp:65-142,180-206; util/bam_deserializer.h:143-193), so the pins are:

* the ranks' records, concatenated in rank order, are byte for byte the records of the whole file as an
  independent host decoder (gzip + the block_size walk, tests/bamutil.py) reads them;
* the sharded mergesort -M chain's output slices concatenate to the one-GPU chain's output;
* every rank decodes only its own blocks (oge_ctx_counter: the blocks sum to the file's, each rank's
  count is its range's).

Edge cases: tiny BGZF blocks (records and the BAM header longer than a rank's part -- the header is
fetched from later ranks, and some parts hold no record start at all), ranges holding no block start,
stored (level-0) blocks with fake BGZF headers planted in the record bytes (false candidates: a wrong
first guess is corrected by the join, a false candidate inside a range takes the host walk), one rank,
and G = 8.  G ranks are G contexts on device 0, one thread each (the in-process transport)."""
import gzip
import struct
import threading
import zlib

import numpy as np
import pytest
import torch

import bamutil
from openge_amd import lib as L

pytestmark = pytest.mark.gpu

FAKE = bytes([31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, ord("B"), ord("C"), 2, 0, 0x3F, 0x00])  # BSIZE 64


def _refs(header):
    out = []
    for line in header.splitlines():
        if line.startswith("@SQ"):
            f = dict(x.split(":", 1) for x in line.split("\t")[1:])
            out.append((f["SN"], int(f["LN"])))
    return out


def _bam_body(header, recs, offs):
    ht = header.encode()
    refs = _refs(header)
    body = b"BAM\1" + struct.pack("<i", len(ht)) + ht + struct.pack("<i", len(refs))
    for name, ln in refs:
        nb = name.encode() + b"\0"
        body += struct.pack("<i", len(nb)) + nb + struct.pack("<i", ln)
    return body + recs[:int(offs[-1])].tobytes()


def _input(pairs, seed, preset="c2", fake_every=0):
    p = L.synth_params(pairs, preset=preset, seed=seed)
    recs, offs, hdr = L.synth_host(p)
    if fake_every:  # fake BGZF headers in the quality bytes of every k-th record (stored blocks show them verbatim)
        for k in range(0, len(offs) - 1, fake_every):
            o = int(offs[k])
            lname, ncig, lseq = int(recs[o + 12]), int(recs[o + 16]) | (int(recs[o + 17]) << 8), int(recs[o + 20:o + 24].view(np.int32)[0])
            q = o + 36 + lname + 4 * ncig + (lseq + 1) // 2
            if lseq >= len(FAKE) + 8:
                recs[q + 4:q + 4 + len(FAKE)] = np.frombuffer(FAKE, np.uint8)
    return recs, offs, hdr


def _records_of(body):
    """the record bytes of a decompressed BAM stream (after the header)"""
    (lt,) = struct.unpack_from("<i", body, 4)
    q = 8 + lt
    (nref,) = struct.unpack_from("<i", body, q)
    q += 4
    for _ in range(nref):
        (ln,) = struct.unpack_from("<i", body, q)
        q += 8 + ln
    return body[q:]


def run_shard(zfile: bytes, G: int, fn):
    """G ranks on device 0 over the file's byte ranges; fn(comm, ctx, d_z, zbytes, own) per rank -> result list"""
    ctxs = [L.Context(0) for _ in range(G)]
    comms = L.comm_init(ctxs)
    res, errs = [None] * G, []
    ranges = L.shard_ranges(len(zfile), G)

    def work(g):
        try:
            a, own, end = ranges[g]
            d_z = torch.from_numpy(np.frombuffer(zfile[a:end] + b"\0" * 64, np.uint8).copy()).cuda()
            torch.cuda.synchronize()
            res[g] = fn(comms[g], ctxs[g], d_z.data_ptr(), end - a, own)
        except Exception as e:  # noqa: BLE001
            errs.append((g, e))

    ts = [threading.Thread(target=work, args=(g,)) for g in range(G)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    for c in comms:
        c.close()
    for c in ctxs:
        c.close()
    if errs:
        raise errs[0][1]
    return res


def _decode(comm, ctx, d_z, zbytes, own):
    dr, do, n, hdr = comm.decode_shard(d_z, zbytes, own)
    oo = np.empty(n + 1, np.uint64)
    L.check(L.lib().oge_memcpy(ctx.h, oo.ctypes.data, do, 8 * (n + 1), 2), ctx.h)
    out = np.empty(int(oo[n] - oo[0]), np.uint8)
    if out.size:
        L.check(L.lib().oge_memcpy(ctx.h, out.ctypes.data, dr + int(oo[0]), out.size, 2), ctx.h)
    # offsets are contiguous: records back to back
    assert np.all(np.diff(oo.astype(np.int64)) > 0) or n == 0
    counts = {k: ctx.counter(k) for k in ("shard_blocks", "shard_zbytes", "shard_bytes", "shard_records")}
    return out.tobytes(), n, hdr, counts


def _blocks_in(zfile, a, b):
    """(BGZF blocks with a payload that start in [a, b), all blocks with a payload) -- host walk"""
    p, mine, tot = 0, 0, 0
    while p < len(zfile):
        bsize = struct.unpack_from("<H", zfile, p + 16)[0] + 1
        isize = struct.unpack_from("<I", zfile, p + bsize - 4)[0]
        if isize:
            tot += 1
            mine += a <= p < b
        p += bsize
    return mine, tot


def _check_decode(zfile, G):
    body = gzip.decompress(zfile)
    want = _records_of(body)
    res = run_shard(zfile, G, _decode)
    got = b"".join(r[0] for r in res)
    assert got == want
    assert sum(r[1] for r in res) == sum(1 for _ in _walk(want))
    hl = len(body) - len(want)
    assert all(r[2] == body[:hl] for r in res)  # every rank has the header
    ranges = L.shard_ranges(len(zfile), G)
    for g, r in enumerate(res):
        a, own, _ = ranges[g]
        mine, tot = _blocks_in(zfile, a, a + own)
        assert r[3]["shard_blocks"] == mine, (g, r[3], mine)
    assert sum(r[3]["shard_bytes"] for r in res) == len(body)
    assert sum(r[3]["shard_zbytes"] for r in res) == len(zfile)
    return res


def _walk(recs: bytes):
    q = 0
    while q < len(recs):
        yield q
        q += 4 + struct.unpack_from("<I", recs, q)[0]


@pytest.mark.parametrize("G", [1, 2, 3, 5, 8])
def test_shard_decode_equals_whole_file(G):
    recs, offs, hdr = _input(30000, 21)
    zfile = bamutil.bgzf_blocks(_bam_body(hdr, recs, offs), level=6)
    res = _check_decode(zfile, G)
    if G > 1:  # the work is split: no rank decodes more than its share (+ one block)
        nb = sum(r[3]["shard_blocks"] for r in res)
        assert max(r[3]["shard_blocks"] for r in res) <= nb // G + 2


@pytest.mark.parametrize("payload,G", [(200, 8), (700, 5), (3000, 3)])
def test_shard_decode_tiny_blocks(payload, G):
    """parts smaller than a record and than the BAM header: some ranks own no record start, rank 0's
    header is fetched from the next ranks' parts"""
    recs, offs, hdr = _input(8, 3)
    body = _bam_body(hdr, recs, offs)
    zfile = bamutil.bgzf_blocks(body, level=1, payload=payload)
    res = _check_decode(zfile, G)
    if payload == 200:
        assert any(r[1] == 0 for r in res)


def test_shard_decode_ranges_without_blocks():
    """3 blocks over 8 ranks: most byte ranges hold no block start"""
    recs, offs, hdr = _input(300, 4)
    zfile = bamutil.bgzf_blocks(_bam_body(hdr, recs, offs), level=6, payload=40000)
    res = _check_decode(zfile, 8)
    assert sum(r[3]["shard_blocks"] == 0 for r in res) >= 3


@pytest.mark.parametrize("fake_every,G", [(7, 4), (31, 8), (1, 3)])
def test_shard_decode_false_block_candidates(fake_every, G):
    """stored blocks with fake BGZF headers inside the records: the candidate scan finds them, the
    framing join rejects them (wrong first guesses corrected, host walk inside a range)"""
    recs, offs, hdr = _input(2000, 9, fake_every=fake_every)
    body = _bam_body(hdr, recs, offs)
    zfile = bamutil.bgzf_blocks(body, level=0, payload=5000)
    assert zfile.count(FAKE) > 0.8 * (len(offs) - 1) / fake_every  # the planted false candidates are in the file
    _check_decode(zfile, G)


@pytest.mark.parametrize("G", [2, 3, 8])
def test_shard_mergesort_equals_one_gpu(ctx, G):
    recs, offs, hdr = _input(40000, 31)
    zfile = bamutil.bgzf_blocks(_bam_body(hdr, recs, offs), level=6)
    mo = L.mergesort_opts(mark_duplicates=1)
    dz = torch.from_numpy(np.frombuffer(zfile + b"\0" * 64, np.uint8).copy()).cuda()
    d, nb, nr, nd = ctx.mergesort_bgzf_dev(dz.data_ptr(), len(zfile), mo)
    h = np.empty(nb, np.uint8)
    L.check(L.lib().oge_memcpy(ctx.h, h.ctypes.data, d, nb, 2), ctx.h)
    want = gzip.decompress(h.tobytes())

    def fn(comm, c, d_z, zbytes, own):
        d2, ob, nr2, nd2 = comm.mergesort_bgzf_shard(d_z, zbytes, own, mo)
        out = np.empty(ob, np.uint8)
        if ob:
            L.check(L.lib().oge_memcpy(c.h, out.ctypes.data, d2, ob, 2), c.h)
        return out.tobytes(), nr2, nd2, comm.exchange_stats()

    res = run_shard(zfile, G, fn)
    out = b"".join(r[0] for r in res)
    assert out[-28:] == bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    assert gzip.decompress(out) == want
    assert all(r[1] == nr and r[2] == nd for r in res)
    tags = {x["tag"] for x in res[0][3]}
    assert {"shard_framing", "shard_edges", "shard_records", "records", "dup_marks"} <= tags
    # the edge exchange moves at most one tail per neighbour (<= 16 KiB each way per rank)
    edges = [x for x in res[0][3] if x["tag"] == "shard_edges"][0]
    assert edges["bytes_recv"] <= 16384


def test_shard_bad_arguments(ctx):
    """own_bytes > zbytes, and a last rank whose buffer stops short of the end: every rank fails"""
    recs, offs, hdr = _input(500, 5)
    zfile = bamutil.bgzf_blocks(_bam_body(hdr, recs, offs), level=6, payload=4000)
    G = 2
    ctxs = [L.Context(0) for _ in range(G)]
    comms = L.comm_init(ctxs)
    errs = [None] * G
    ranges = L.shard_ranges(len(zfile), G)

    def work(g):
        a, own, end = ranges[g]
        if g == G - 1:
            end -= 10  # truncated
        d_z = torch.from_numpy(np.frombuffer(zfile[a:end] + b"\0" * 64, np.uint8).copy()).cuda()
        torch.cuda.synchronize()
        try:
            comms[g].decode_shard(d_z.data_ptr(), end - a, min(own, end - a))
        except Exception as e:  # noqa: BLE001
            errs[g] = str(e)

    ts = [threading.Thread(target=work, args=(g,)) for g in range(G)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    for c in comms:
        c.close()
    for c in ctxs:
        c.close()
    assert all(errs), errs
