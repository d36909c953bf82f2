"""GPU: multi-GPU sort + duplicate marking through the C ABI (oge_comm_init / oge_sort_markdup_dist,
openge_amd/csrc/dist.hip) equals the one-GPU `mergesort [-M] --nosplit` output record for record.

On the one-GPU test box G ranks are G contexts on device 0, one thread each, joined by the
in-process transport (the same schedule RCCL runs between GPUs).  Inputs: the reference-made golden
cases, C2/mix synthetic sets, and C2 with supplementary (0x800, counted as primary by the reference,
bt/BamAlignment.cpp:493-495) copies on other contigs, so names carry 3 and 4 primaries whose
ReadEndsMap pairing (mark_duplicates.cpp:213-245) depends on the global order of their ends --
checked against the oracle restatement as well.  Shards are contiguous input ranges (one of them
empty in one case) and, separately, an interleaved split."""
import struct
import threading

import numpy as np
import pytest
import torch

import bamutil
import oracle
from goldens import CASE_NAMES, load_case
from openge_amd import lib as L

pytestmark = pytest.mark.gpu


def _single(ctx, recs, offs, n, n_ref, opts):
    d_recs = torch.from_numpy(recs).cuda()
    d_offs = torch.from_numpy(offs.astype(np.int64)).cuda()
    d_perm = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
    d_out = torch.empty(recs.size, dtype=torch.uint8, device="cuda")
    d_oo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    nd = 0
    if opts is not None:
        nd = ctx.sort_markdup_dev(d_recs.data_ptr(), d_offs.data_ptr(), n, opts, d_perm.data_ptr(), d_out.data_ptr(),
                                  d_oo.data_ptr())
    else:
        ctx.sort_coord_dev(d_recs.data_ptr(), d_offs.data_ptr(), n, n_ref, d_perm.data_ptr())
        ctx.gather_records_dev(d_recs.data_ptr(), d_offs.data_ptr(), d_perm.data_ptr(), n, d_out.data_ptr(), d_oo.data_ptr())
    ctx.sync()
    oo = d_oo.cpu().numpy()
    return d_out[int(oo[0]):int(oo[n])].cpu().numpy().tobytes(), nd


def _shards(recs, offs, cuts):
    """contiguous input ranges [cuts[g], cuts[g+1]) as (record bytes, offsets from 0)"""
    out = []
    for g in range(len(cuts) - 1):
        lo, hi = cuts[g], cuts[g + 1]
        b0, b1 = int(offs[lo]), int(offs[hi])
        out.append((np.concatenate([recs[b0:b1], np.zeros(64, np.uint8)]), (offs[lo:hi + 1] - b0).astype(np.int64)))
    return out


def run_dist(shards, n_ref, opts, sort=True):
    """One rank per shard, all on device 0; returns (concatenated output stream, per-rank counts, dups)."""
    G = len(shards)
    ctxs = [L.Context(0) for _ in range(G)]
    comms = L.comm_init(ctxs)
    assert comms[0].transport == "local" and comms[0].size == G
    res, errs = [None] * G, []

    def work(g):
        try:
            recs, offs = shards[g]
            n = len(offs) - 1
            d_recs = torch.from_numpy(recs).cuda()
            d_offs = torch.from_numpy(offs).cuda()
            torch.cuda.synchronize()
            d, do, no, nd = comms[g].sort_markdup_dist(d_recs.data_ptr(), d_offs.data_ptr(), n, n_ref, opts, sort)
            oo = np.empty(no + 1, np.uint64)
            L.check(L.lib().oge_memcpy(ctxs[g].h, oo.ctypes.data, do, 8 * (no + 1), 2), ctxs[g].h)
            out = np.empty(int(oo[no] - oo[0]), np.uint8)
            if out.size:
                L.check(L.lib().oge_memcpy(ctxs[g].h, out.ctypes.data, d + int(oo[0]), out.size, 2), ctxs[g].h)
            res[g] = (out.tobytes(), no, nd)
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
    assert len({r[2] for r in res}) == 1  # every rank reports the same total
    return b"".join(r[0] for r in res), [r[1] for r in res], res[0][2]


def _check(ctx, recs, offs, n_ref, header, G, cuts=None, sort_only=False):
    n = len(offs) - 1
    opts = None
    if not sort_only:
        opts, keep = L.markdup_opts_from_header(header, n_ref)
    want, nd = _single(ctx, recs, offs, n, n_ref, opts)
    cuts = cuts or [n * g // G for g in range(G + 1)]
    got, counts, gd = run_dist(_shards(recs, offs, cuts), n_ref, opts)
    assert sum(counts) == n
    assert got == want
    assert gd == nd
    return counts, nd


@pytest.mark.parametrize("name", CASE_NAMES)
@pytest.mark.parametrize("G", [2, 3])
def test_dist_equals_single_on_goldens(ctx, name, G):
    c = load_case(name)
    _check(ctx, c.recs, c.offs, c.n_ref, c.header, G)
    if G == 3:  # sort only (mergesort without -M)
        _check(ctx, c.recs, c.offs, c.n_ref, c.header, G, sort_only=True)


@pytest.mark.parametrize("preset,pairs,seed,G", [("c2", 40000, 11, 2), ("c2", 40000, 12, 3), ("mix", 6000, 5, 3),
                                                  ("c2", 60000, 13, 5), ("c2", 40000, 14, 4), ("c2", 60000, 15, 8)])
def test_dist_equals_single_synthetic(ctx, preset, pairs, seed, G):
    p = L.synth_params(pairs, preset=preset, seed=seed)
    recs, offs, hdr = L.synth_host(p)
    counts, nd = _check(ctx, recs, offs, p.n_ref, hdr, G)
    assert nd > 0
    if preset == "c2":  # range splitters balance the slices (sampling error only)
        assert max(counts) / (sum(counts) / G) < 1.05


def test_dist_uneven_and_empty_shards(ctx):
    p = L.synth_params(8000, preset="c2", seed=21)
    recs, offs, hdr = L.synth_host(p)
    n = len(offs) - 1
    _check(ctx, recs, offs, p.n_ref, hdr, 3, cuts=[0, 0, n // 5, n])
    _check(ctx, recs, offs, p.n_ref, hdr, 2, cuts=[0, n, n])


def _with_supplementaries(recs, offs, n_ref, ref_len, seed):
    """C2 records plus 0x800 copies of ~4% of the reads on another contig (a few names get two),
    mate fields unchanged: 3- and 4-primary names for the ReadEndsMap."""
    rng = np.random.default_rng(seed)
    n = len(offs) - 1
    out = [bamutil.rec_bytes(recs, offs[i]) for i in range(n)]
    pick = rng.choice(n, size=n // 25, replace=False)
    extra = []
    for k, i in enumerate(pick):
        for _ in range(2 if k % 7 == 0 else 1):
            b = bytearray(out[i])
            (flag,) = struct.unpack_from("<H", b, 18)
            ref = int(rng.integers(0, n_ref))
            pos = int(rng.integers(0, max(1, ref_len[ref] - 200)))
            struct.pack_into("<iI", b, 4, ref, pos)
            struct.pack_into("<H", b, 18, (flag | 0x800) & ~0x400)
            extra.append(bytes(b))
    allr = out + extra
    order = rng.permutation(len(allr))
    return bamutil.pack_records([allr[j] for j in order])


@pytest.mark.parametrize("G", [2, 3])
def test_dist_supplementary_names_exact(ctx, G):
    p = L.synth_params(15000, preset="c2", seed=31)
    recs0, offs0, hdr = L.synth_host(p)
    lens = [int(p.ref_len[i]) for i in range(p.n_ref)]
    recs, offs = _with_supplementaries(recs0, offs0, p.n_ref, lens, 32)
    n = len(offs) - 1
    # the one-GPU path against the oracle restatement of mark_duplicates.cpp on the sorted stream
    perm = oracle.sort_perm(recs, offs, n)
    srecs, soffs = bamutil.pack_records([bamutil.rec_bytes(recs, offs[i]) for i in perm])
    opts, keep = L.markdup_opts_from_header(hdr, p.n_ref)
    dup, nd = ctx.markdup(srecs, soffs, n, opts)
    odup, ond = oracle.markdup(srecs, soffs, n, hdr)
    assert nd == ond and np.array_equal(dup, odup)
    # the multi-GPU path against the one-GPU path, contiguous and interleaved input splits
    _check(ctx, recs, offs, p.n_ref, hdr, G)
    inter = np.concatenate([np.arange(g, n, G) for g in range(G)])
    irecs, ioffs = bamutil.pack_records([bamutil.rec_bytes(recs, offs[i]) for i in inter])
    _check(ctx, irecs, ioffs, p.n_ref, hdr, G)


def _unbin(stream: bytes) -> bytes:
    """the record stream with every bin field zeroed (dedup leaves bins as read; the gather recomputes)"""
    b, q = bytearray(stream), 0
    while q < len(b):
        (bs,) = struct.unpack_from("<I", b, q)
        b[q + 14:q + 16] = b"\0\0"
        q += 4 + bs
    return bytes(b)


@pytest.mark.parametrize("name,G", [("yhet208", 2), ("c2_20k", 3), ("mix3k", 2), ("edge", 3)])
def test_dist_dedup_keeps_input_order(ctx, name, G):
    """`dedup --gpus G`: each rank marks its input shard in place order, exactly as one GPU marks the
    whole stream (oge_markdup_dev, record index = input position)."""
    c = load_case(name)
    opts, keep = L.markdup_opts_from_header(c.header, c.n_ref)
    d_recs = torch.from_numpy(c.recs.copy()).cuda()
    d_offs = torch.from_numpy(c.offs.astype(np.int64)).cuda()
    d_dup = torch.empty(c.n + 1, dtype=torch.uint8, device="cuda")
    nd = ctx.markdup_dev(d_recs.data_ptr(), d_offs.data_ptr(), c.n, opts, d_dup.data_ptr(), apply=1)
    ctx.sync()
    want = d_recs[int(c.offs[0]):int(c.offs[c.n])].cpu().numpy().tobytes()
    got, counts, gd = run_dist(_shards(c.recs, c.offs, [c.n * g // G for g in range(G + 1)]), c.n_ref, opts, sort=False)
    assert gd == nd and sum(counts) == c.n
    assert _unbin(got) == _unbin(want)


@pytest.mark.parametrize("G,level,flags", [(2, 6, {"mark_duplicates": 1}), (3, 1, {"mark_duplicates": 1, "remove_duplicates": 1}),
                                           (2, 6, {})])
def test_dist_bgzf_chain_equals_single(ctx, tmp_path, G, level, flags):
    """oge_mergesort_bgzf_dist: G input BAM files (contiguous ranges of one input, same header) -> G
    output slices that concatenate into one BAM file whose decompressed bytes equal the one-GPU
    oge_mergesort_bgzf_dev output's."""
    import gzip
    p = L.synth_params(30000, preset="c2", seed=41)
    recs, offs, hdr = L.synth_host(p)
    n = len(offs) - 1
    src = tmp_path / "all.bam"
    L.write_bam(src, hdr, recs, offs, n, level=1)
    z = src.read_bytes()
    opts = L.mergesort_opts(level=level, program_line=b"openge mergesort x", **flags)
    dz = torch.from_numpy(np.frombuffer(z + b"\0" * 8, np.uint8).copy()).cuda()
    d, nb, nr, nd = ctx.mergesort_bgzf_dev(dz.data_ptr(), len(z), opts)
    want = np.empty(nb, np.uint8)
    L.check(L.lib().oge_memcpy(ctx.h, want.ctypes.data, d, nb, 2), ctx.h)
    files = []
    for g in range(G):
        lo, hi = n * g // G, n * (g + 1) // G
        fg = tmp_path / f"part{g}.bam"
        r0, r1 = int(offs[lo]), int(offs[hi])
        part = np.concatenate([recs[r0:r1], np.zeros(16, np.uint8)])
        L.write_bam(fg, hdr, part, (offs[lo:hi + 1] - r0).astype(np.uint64), hi - lo, level=1)
        files.append(fg.read_bytes())
    ctxs = [L.Context(0) for _ in range(G)]
    comms = L.comm_init(ctxs)
    res, errs = [None] * G, []

    def work(g):
        try:
            b = files[g]
            t = torch.from_numpy(np.frombuffer(b + b"\0" * 8, np.uint8).copy()).cuda()
            torch.cuda.synchronize()
            d, ob, tr, td = comms[g].mergesort_bgzf_dist(t.data_ptr(), len(b), opts)
            h = np.empty(ob, np.uint8)
            L.check(L.lib().oge_memcpy(ctxs[g].h, h.ctypes.data, d, ob, 2), ctxs[g].h)
            res[g] = (h.tobytes(), tr, td)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

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
        raise errs[0]
    out = b"".join(r[0] for r in res)
    assert out[-28:] == bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    assert gzip.decompress(out) == gzip.decompress(want.tobytes())
    assert {(r[1], r[2]) for r in res} == {(nr, nd)}


def _pile(recs, offs, frac, seed):
    """C2 records with a fraction moved onto ONE coordinate (refID 0, pos 1000, forward strand): a
    uniform-key pile.  Equal ByPosition keys never straddle ranks, so the splitters degenerate -- with
    frac = 1 every record has the same key and all of them land on one rank, the others get nothing."""
    rng = np.random.default_rng(seed)
    n = len(offs) - 1
    out = [bytearray(bamutil.rec_bytes(recs, offs[i])) for i in range(n)]
    pick = np.arange(n) if frac >= 1 else rng.choice(n, size=int(n * frac), replace=False)
    for i in pick:
        b = out[i]
        (flag,) = struct.unpack_from("<H", b, 18)
        struct.pack_into("<iI", b, 4, 0, 1000)
        struct.pack_into("<H", b, 18, flag & ~0x10 & ~0x400)
    return bamutil.pack_records([bytes(b) for b in out])


@pytest.mark.parametrize("frac,G", [(0.6, 8), (1.0, 8), (1.0, 4)])
def test_dist_uniform_key_pile(ctx, frac, G):
    """Splitter degeneracy at the node's rank counts: a pile of identical ByPosition keys (60% of the
    reads, then all of them).  The one-GPU marks are pinned to the oracle restatement first (the pile
    takes the windowed dedup's overflow path), then the G-rank output must equal the one-GPU output."""
    p = L.synth_params(6000, preset="c2", seed=51)
    recs0, offs0, hdr = L.synth_host(p)
    recs, offs = _pile(recs0, offs0, frac, 52)
    n = len(offs) - 1
    perm = oracle.sort_perm(recs, offs, n)
    srecs, soffs = bamutil.pack_records([bamutil.rec_bytes(recs, offs[i]) for i in perm])
    opts, keep = L.markdup_opts_from_header(hdr, p.n_ref)
    dup, nd = ctx.markdup(srecs, soffs, n, opts)
    odup, ond = oracle.markdup(srecs, soffs, n, hdr)
    assert nd == ond and np.array_equal(dup, odup)
    counts, nd2 = _check(ctx, recs, offs, p.n_ref, hdr, G)
    assert nd2 == nd
    if frac >= 1:  # one rank holds the whole pile
        assert sorted(counts)[-1] == n and sum(1 for c in counts if c) == 1


@pytest.mark.parametrize("sort,hostx", [(True, False), (False, False), (True, True), (False, True)])
def test_rccl_transport_world1(ctx, sort, hostx, monkeypatch, tmp_path):
    """RcclTransport's three methods on the one-GPU box: a one-rank communicator forced onto RCCL
    (oge_comm_init_rank_mode "rccl": ncclCommInitRank with one rank) runs the whole distributed step --
    all-to-all-v as grouped ncclSend / ncclRecv to itself, the plans and samples gathered, ncclReduceScatter
    (max) for the marks -- and must equal the one-GPU output (sort + dedup, and the in-place dedup mode).
    hostx: the launcher says every rank is on this node (LOCAL_WORLD_SIZE), so the statuses, plans and
    samples go through the node's shared segment ("host_memory"); else through ncclAllGather and a device
    round trip.  More ranks need more GPUs (RCCL refuses two ranks on one device)."""
    monkeypatch.setenv("OGE_COMM_DIR", str(tmp_path))
    for v in ("LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS", "SLURM_NTASKS_PER_NODE",
              "SLURM_STEP_TASKS_PER_NODE"):
        monkeypatch.delenv(v, raising=False)
    if hostx:
        monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    p = L.synth_params(20000, preset="c2", seed=31)
    recs, offs, hdr = L.synth_host(p)
    n = len(offs) - 1
    opts, keep = L.markdup_opts_from_header(hdr, p.n_ref)
    c1 = L.Context(0)
    comm = L.comm_init_rank(c1, 1, 0, L.comm_unique_id(), mode="rccl")
    try:
        assert comm.transport == "rccl" and comm.size == 1
        (srecs, soffs), = _shards(recs, offs, [0, n])
        d_recs = torch.from_numpy(srecs).cuda()
        d_offs = torch.from_numpy(soffs).cuda()
        torch.cuda.synchronize()
        d, do, no, nd = comm.sort_markdup_dist(d_recs.data_ptr(), d_offs.data_ptr(), n, p.n_ref, opts, sort)
        assert no == n and nd > 0
        oo = np.empty(no + 1, np.uint64)
        L.check(L.lib().oge_memcpy(c1.h, oo.ctypes.data, do, 8 * (no + 1), 2), c1.h)
        got = np.empty(int(oo[no] - oo[0]), np.uint8)
        L.check(L.lib().oge_memcpy(c1.h, got.ctypes.data, d + int(oo[0]), got.size, 2), c1.h)
        ex = {e["tag"]: e for e in comm.exchange_stats()}
        assert ex and all(e["calls"] >= 1 for e in ex.values())
        assert ex["status"]["mode"] == ("host_memory" if hostx else "device_round_trip")
        assert ex["plans"]["mode"] == ex["status"]["mode"]
    finally:
        comm.close()
        c1.close()
    if sort:
        want, wd = _single(ctx, recs, offs, n, p.n_ref, opts)
        assert got.tobytes() == want and nd == wd
    else:  # dedup mode: the input order, the same marks as the in-process two-rank run
        want, counts, wd = run_dist(_shards(recs, offs, [0, n // 2, n]), p.n_ref, opts, sort=False)
        assert got.tobytes() == want and nd == wd


def test_rccl_transport_world1_bgzf_chain(ctx, tmp_path):
    """bench.py --gpus N's call (oge_mergesort_bgzf_dist) over a one-rank RCCL communicator: the output
    file inflates to the one-GPU chain's bytes, with the same record and duplicate counts."""
    import gzip
    p = L.synth_params(20000, preset="c2", seed=43)
    recs, offs, hdr = L.synth_host(p)
    n = len(offs) - 1
    src = tmp_path / "all.bam"
    L.write_bam(src, hdr, recs, offs, n, level=1)
    z = src.read_bytes()
    opts = L.mergesort_opts(level=6, program_line=b"openge mergesort x", mark_duplicates=1)
    dz = torch.from_numpy(np.frombuffer(z + b"\0" * 8, np.uint8).copy()).cuda()
    d, nb, nr, nd = ctx.mergesort_bgzf_dev(dz.data_ptr(), len(z), opts)
    want = np.empty(nb, np.uint8)
    L.check(L.lib().oge_memcpy(ctx.h, want.ctypes.data, d, nb, 2), ctx.h)
    c1 = L.Context(0)
    comm = L.comm_init_rank(c1, 1, 0, L.comm_unique_id(), mode="rccl")
    try:
        assert comm.transport == "rccl"
        t = torch.from_numpy(np.frombuffer(z + b"\0" * 8, np.uint8).copy()).cuda()
        torch.cuda.synchronize()
        d2, ob, tr, td = comm.mergesort_bgzf_dist(t.data_ptr(), len(z), opts)
        got = np.empty(ob, np.uint8)
        L.check(L.lib().oge_memcpy(c1.h, got.ctypes.data, d2, ob, 2), c1.h)
    finally:
        comm.close()
        c1.close()
    assert (tr, td) == (nr, nd)
    assert gzip.decompress(got.tobytes()) == gzip.decompress(want.tobytes())


def test_rccl_transport_world1_shard_chain(ctx, tmp_path):
    """bench.py --gpus N's call since r05 (oge_mergesort_bgzf_shard: ONE file, ranks decode their byte
    ranges) over a one-rank RCCL communicator: the framing and record joins (ncclAllGather), the tail
    fetch (grouped ncclSend / ncclRecv) and the sort + dedup step equal the one-GPU chain."""
    import gzip
    p = L.synth_params(20000, preset="c2", seed=47)
    recs, offs, hdr = L.synth_host(p)
    n = len(offs) - 1
    src = tmp_path / "all.bam"
    L.write_bam(src, hdr, recs, offs, n, level=6)
    z = src.read_bytes()
    opts = L.mergesort_opts(level=6, mark_duplicates=1)
    dz = torch.from_numpy(np.frombuffer(z + b"\0" * 8, np.uint8).copy()).cuda()
    d, nb, nr, nd = ctx.mergesort_bgzf_dev(dz.data_ptr(), len(z), opts)
    want = np.empty(nb, np.uint8)
    L.check(L.lib().oge_memcpy(ctx.h, want.ctypes.data, d, nb, 2), ctx.h)
    c1 = L.Context(0)
    comm = L.comm_init_rank(c1, 1, 0, L.comm_unique_id(), mode="rccl")
    try:
        assert comm.transport == "rccl"
        t = torch.from_numpy(np.frombuffer(z + b"\0" * 8, np.uint8).copy()).cuda()
        torch.cuda.synchronize()
        d2, ob, tr, td = comm.mergesort_bgzf_shard(t.data_ptr(), len(z), len(z), opts)
        got = np.empty(ob, np.uint8)
        L.check(L.lib().oge_memcpy(c1.h, got.ctypes.data, d2, ob, 2), c1.h)
    finally:
        comm.close()
        c1.close()
    assert (tr, td) == (nr, nd)
    assert gzip.decompress(got.tobytes()) == gzip.decompress(want.tobytes())


def test_rccl_transport_world1_blocking_records(ctx, monkeypatch):
    """The blocking record exchange (OGE_DIST_RECORDS=blocking) over a one-rank RCCL communicator: the
    records themselves go through grouped ncclSend / ncclRecv (to the rank itself: the side-stream mode
    moves only peers' parts through the transport), non-zero bytes, and the output equals one GPU's."""
    monkeypatch.setenv("OGE_DIST_RECORDS", "blocking")
    p = L.synth_params(20000, preset="c2", seed=53)
    recs, offs, hdr = L.synth_host(p)
    n = len(offs) - 1
    opts, keep = L.markdup_opts_from_header(hdr, p.n_ref)
    c1 = L.Context(0)
    comm = L.comm_init_rank(c1, 1, 0, L.comm_unique_id(), mode="rccl")
    try:
        (srecs, soffs), = _shards(recs, offs, [0, n])
        d_recs = torch.from_numpy(srecs).cuda()
        d_offs = torch.from_numpy(soffs).cuda()
        torch.cuda.synchronize()
        d, do, no, nd = comm.sort_markdup_dist(d_recs.data_ptr(), d_offs.data_ptr(), n, p.n_ref, opts, True)
        oo = np.empty(no + 1, np.uint64)
        L.check(L.lib().oge_memcpy(c1.h, oo.ctypes.data, do, 8 * (no + 1), 2), c1.h)
        got = np.empty(int(oo[no] - oo[0]), np.uint8)
        L.check(L.lib().oge_memcpy(c1.h, got.ctypes.data, d + int(oo[0]), got.size, 2), c1.h)
        ex = {e["tag"]: e for e in comm.exchange_stats()}
    finally:
        comm.close()
        c1.close()
    want, wd = _single(ctx, recs, offs, n, p.n_ref, opts)
    assert got.tobytes() == want and nd == wd
    rec = ex["records"]
    assert rec["calls"] >= 1 and rec["mode"] == "blocking" and rec["bytes_self"] > 0
    # r06: RCCL collectives are stream-ordered and not waited for; their time comes from HIP events around them
    assert rec["device_ms"] > 0 and ex["dup_marks"]["device_ms"] > 0
    print("records exchange over RCCL at world 1:", rec)
