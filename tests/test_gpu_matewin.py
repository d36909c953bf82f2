"""GPU: the windowed mate join of the fused sort + dedup (markdup.hip k_mate_win / k_mate_agree /
k_mate_check + the sort-based join for the leftovers) against the sort-based join alone
(OGE_MD_MATEWIN=0) and the oracle restatement of MarkDuplicates (mark_duplicates.cpp:185-245, pairing of
consecutive occurrences of each RG:name key), on inputs whose mates sit outside the window, whose names
occur more than twice (supplementary records) and whose pairs cross contigs."""
import numpy as np
import pytest
import torch

import bamutil
import oracle
from openge_amd import lib as L
from test_gpu_dist import _with_supplementaries

pytestmark = pytest.mark.gpu


def _fused(ctx, recs, offs, n, opts):
    d_recs = torch.from_numpy(recs.copy()).cuda()
    d_offs = torch.from_numpy(offs[:n + 1].astype(np.int64)).cuda()
    tot = int(offs[n] - offs[0])
    d_perm = torch.empty(n, dtype=torch.int32, device="cuda")
    d_out = torch.empty(tot + 64, dtype=torch.uint8, device="cuda")
    d_oo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    nd = ctx.sort_markdup_dev(d_recs.data_ptr(), d_offs.data_ptr(), n, opts, d_perm.data_ptr(), d_out.data_ptr(), d_oo.data_ptr())
    ctx.sync()
    return nd, d_out[:tot].cpu().numpy().tobytes(), {k: ctx.counter(k) for k in ("md_mate_left", "md_mate_pairs",
                                                                                   "md_mate_redo", "md_mate_ovf")}


def _both(ctx, monkeypatch, recs, offs, hdr, n_ref):
    n = len(offs) - 1
    opts, keep = L.markdup_opts_from_header(hdr, n_ref)
    monkeypatch.setenv("OGE_MD_MATEWIN", "0")
    nd0, out0, _ = _fused(ctx, recs, offs, n, opts)
    monkeypatch.delenv("OGE_MD_MATEWIN")
    nd1, out1, c = _fused(ctx, recs, offs, n, opts)
    assert nd1 == nd0 and out1 == out0
    return nd1, c


@pytest.mark.parametrize("ins_max", [450, 3000, 20000])
def test_window_join_equals_sort_join(ctx, monkeypatch, ins_max):
    # one short contig, dense reads: mates 100s to 1000s of records apart (the window is 512 each side)
    p = L.synth_params(400_000, preset="c2", seed=77, ins_max=ins_max, n_ref=1, ref_len=[2_000_000])
    recs, offs, hdr = L.synth_host(p, threads=8)
    nd, c = _both(ctx, monkeypatch, recs, offs, hdr, p.n_ref)
    assert nd > 0 and not c["md_mate_redo"]
    if ins_max == 450:
        assert c["md_mate_pairs"] > 0 and not c["md_mate_ovf"]
    else:  # many mates outside the window: the leftovers took the sort path, or overflowed the set (all by sort)
        assert c["md_mate_left"] > 1000


def test_window_join_supplementaries_and_contigs(ctx, monkeypatch):
    p = L.synth_params(20000, preset="c2", seed=31)
    recs0, offs0, hdr = L.synth_host(p)
    lens = [int(p.ref_len[i]) for i in range(p.n_ref)]
    recs, offs = _with_supplementaries(recs0, offs0, p.n_ref, lens, 32)
    nd, c = _both(ctx, monkeypatch, recs, offs, hdr, p.n_ref)
    assert c["md_mate_left"] > 0 and c["md_mate_pairs"] > 0
    # and the oracle on the sorted stream
    n = len(offs) - 1
    perm = oracle.sort_perm(recs, offs, n)
    srecs, soffs = bamutil.pack_records([bamutil.rec_bytes(recs, offs[i]) for i in perm])
    _, ond = oracle.markdup(srecs, soffs, n, hdr)
    assert nd == ond


def test_window_join_c2_counts(ctx, monkeypatch):
    p = L.synth_params(300_000, preset="c2", seed=5)
    recs, offs, hdr = L.synth_host(p, threads=8)
    nd, c = _both(ctx, monkeypatch, recs, offs, hdr, p.n_ref)
    n = len(offs) - 1
    # inter-contig pairs (1%) and pairs with an unmapped mate are the leftovers; most pairs are windowed
    assert c["md_mate_left"] < 0.05 * n and c["md_mate_pairs"] > 0.4 * n


def _offsets(buf: np.ndarray, n: int) -> np.ndarray:
    """record start offsets (n + 1) of a packed record stream, by its block_size fields"""
    offs = np.empty(n + 1, dtype=np.uint64)
    o, b = 0, buf.tobytes()
    for i in range(n):
        offs[i] = o
        o += 4 + int.from_bytes(b[o:o + 4], "little")
    offs[n] = o
    return offs


def _inplace(ctx, recs, offs, n, opts):
    """oge_markdup_dev in place (`openge dedup`: record index = input position) -> (nd, dup bytes, records
    after apply, whether the windowed paths ran)."""
    d_recs = torch.from_numpy(recs.copy()).cuda()
    d_offs = torch.from_numpy(offs[:n + 1].astype(np.int64)).cuda()
    d_dup = torch.empty(n + 1, dtype=torch.uint8, device="cuda")
    nd = ctx.markdup_dev(d_recs.data_ptr(), d_offs.data_ptr(), n, opts, d_dup.data_ptr(), apply=True)
    ctx.sync()
    return nd, d_dup[:n].cpu().numpy(), d_recs.cpu().numpy().tobytes(), ctx.counter("md_inplace_window")


@pytest.mark.parametrize("preset,pairs,kw", [("c2", 300_000, {}), ("mix", 40_000, {}),
                                             ("c2", 200_000, {"ins_max": 3000, "n_ref": 1, "ref_len": [2_000_000]})])
def test_inplace_dedup_window_on_sorted_input(ctx, monkeypatch, preset, pairs, kw):
    """`openge dedup` on a coordinate-sorted file: the in-place path verifies the input's
    anchors never decrease and then takes the windowed mate join and groups -- the same marks and records as
    its sort-based paths (OGE_MD_INPLACE_WINDOW=0), as the fused chain's marks, and as the oracle."""
    p = L.synth_params(pairs, preset=preset, seed=2468, **kw)
    recs, offs, hdr = L.synth_host(p, threads=8)
    n = len(offs) - 1
    opts, keep = L.markdup_opts_from_header(hdr, p.n_ref)
    nd_f, sorted_bytes, _ = _fused(ctx, recs, offs, n, opts)  # sorted records, 0x400 already applied
    srecs = np.frombuffer(sorted_bytes, np.uint8).copy()
    soffs = _offsets(srecs, n)
    nd1, dup1, out1, win = _inplace(ctx, srecs, soffs, n, opts)
    assert win == 1
    monkeypatch.setenv("OGE_MD_INPLACE_WINDOW", "0")
    nd0, dup0, out0, win0 = _inplace(ctx, srecs, soffs, n, opts)
    monkeypatch.delenv("OGE_MD_INPLACE_WINDOW")
    assert not win0
    assert nd1 == nd0 == nd_f and np.array_equal(dup1, dup0) and out1 == out0
    assert out1 == sorted_bytes  # apply on the fused output reproduces its own 0x400 bits
    odup, ond = oracle.markdup(srecs, soffs[:-1], n, hdr)
    sure = odup != 2
    assert np.array_equal(dup1[sure].astype(bool), odup[sure].astype(bool)) and nd1 == ond


def test_inplace_dedup_unsorted_input_keeps_sort_paths(ctx):
    """Input order (not coordinate-sorted): the anchor check fails, the sort-based paths run, and the marks
    equal the oracle's."""
    p = L.synth_params(30_000, preset="mix", seed=99)
    recs, offs, hdr = L.synth_host(p)
    n = len(offs) - 1
    opts, keep = L.markdup_opts_from_header(hdr, p.n_ref)
    nd, dup, _, win = _inplace(ctx, recs, offs, n, opts)
    assert win == 0
    odup, ond = oracle.markdup(recs, offs[:-1], n, hdr)
    sure = odup != 2
    assert np.array_equal(dup[sure].astype(bool), odup[sure].astype(bool)) and nd == ond
