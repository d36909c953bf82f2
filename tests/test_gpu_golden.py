"""GPU: the HIP path against the REFERENCE's own outputs (tests/golden, made by oracle/_ref)."""
import hashlib

import numpy as np
import pytest

import bamutil
from goldens import CASE_NAMES, check_dups, check_perm, load_case
from openge_amd import lib as L

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=CASE_NAMES)
def case(request, built):
    return load_case(request.param)


def test_gpu_sort_matches_reference(ctx, case):
    perm = ctx.sort_coord(case.recs, case.offs, case.n, case.n_ref)
    check_perm(case, perm)


def test_gpu_dedup_matches_reference(ctx, case):
    opts, keep = L.markdup_opts_from_header(case.header, case.n_ref)
    perm = ctx.sort_coord(case.recs, case.offs, case.n, case.n_ref)
    srecs, soffs = bamutil.pack_records([bamutil.rec_bytes(case.recs, case.offs[i]) for i in perm])
    dup, _ = ctx.markdup(srecs, soffs, case.n, opts)
    check_dups(case, "dedup_sorted_v", dup, case.offs[:-1][perm])
    dup, _ = ctx.markdup(case.recs, case.offs, case.n, opts)
    check_dups(case, "dedup_input_v", dup, case.offs)
    o2, keep2 = L.markdup_opts_from_header(case.header, case.n_ref, compat_nonverbose=True)
    dup, _ = ctx.markdup(case.recs, case.offs, case.n, o2)
    check_dups(case, "dedup_input_nv", dup, case.offs)


@pytest.mark.parametrize("k", [3, 12])
def test_gpu_dedup_split_chains(ctx, case, k):
    """split-by-chromosome emulation (mates in different refID % K chains never pair)."""
    opts, keep = L.markdup_opts_from_header(case.header, case.n_ref, split_chains=k)
    perm = ctx.sort_coord(case.recs, case.offs, case.n, case.n_ref)
    srecs, soffs = bamutil.pack_records([bamutil.rec_bytes(case.recs, case.offs[i]) for i in perm])
    dup, _ = ctx.markdup(srecs, soffs, case.n, opts)
    check_dups(case, f"dedup_sorted_v_k{k}", dup, case.offs[:-1][perm])


def test_gpu_split_chains_reject_nonverbose(ctx, case):
    opts, keep = L.markdup_opts_from_header(case.header, case.n_ref, compat_nonverbose=True, split_chains=3)
    with pytest.raises(L.OgeError, match="split_chains"):
        ctx.markdup(case.recs, case.offs, case.n, opts)


def test_gpu_fused_stream_is_reference_bytes(ctx, case):
    """sort + markdup on device: the output record stream (bin recomputed, 0x400 applied) equals the
    reference `mergesort -M` output byte for byte (mapped records in order; unmapped tail as multiset)."""
    torch = pytest.importorskip("torch")
    n, tot = case.n, int(case.offs[-1])
    d_recs = torch.from_numpy(case.recs).cuda()
    d_offs = torch.from_numpy(case.offs.view(np.int64)).cuda()
    d_perm = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
    d_out = torch.zeros(tot + 16, dtype=torch.uint8, device="cuda")
    d_out_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    opts, keep = L.markdup_opts_from_header(case.header, case.n_ref)
    ctx.sort_markdup_dev(d_recs.data_ptr(), d_offs.data_ptr(), n, opts, d_perm.data_ptr(), d_out.data_ptr(),
                         d_out_off.data_ptr())
    ctx.sync()
    out = d_out.cpu().numpy()
    oo = d_out_off.cpu().numpy().view(np.uint64)
    h, tail = hashlib.sha256(), []
    for k in range(n):
        rb = bamutil.rec_bytes(out, oo[k])
        (tail.append(rb) if int.from_bytes(rb[4:8], "little", signed=True) == -1 else h.update(rb))
    g = case.meta["sortdedup_v"]
    assert h.hexdigest() == g["mapped_sha256"]
    assert hashlib.sha256(b"".join(sorted(tail))).hexdigest() == g["tail_multiset_sha256"]


def test_gpu_fused_split_stream_is_reference_bytes(ctx, case):
    """`mergesort -M` with the reference's default split chains (K = 3) on device, byte for byte."""
    torch = pytest.importorskip("torch")
    n, tot = case.n, int(case.offs[-1])
    d_recs = torch.from_numpy(case.recs).cuda()
    d_offs = torch.from_numpy(case.offs.view(np.int64)).cuda()
    d_perm = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
    d_out = torch.zeros(tot + 16, dtype=torch.uint8, device="cuda")
    d_out_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    opts, keep = L.markdup_opts_from_header(case.header, case.n_ref, split_chains=3)
    ctx.sort_markdup_dev(d_recs.data_ptr(), d_offs.data_ptr(), n, opts, d_perm.data_ptr(), d_out.data_ptr(),
                         d_out_off.data_ptr())
    ctx.sync()
    out = d_out.cpu().numpy()
    oo = d_out_off.cpu().numpy().view(np.uint64)
    h, tail = hashlib.sha256(), []
    for k in range(n):
        rb = bamutil.rec_bytes(out, oo[k])
        (tail.append(rb) if int.from_bytes(rb[4:8], "little", signed=True) == -1 else h.update(rb))
    g = case.meta["sortdedup_v_k3"]
    assert h.hexdigest() == g["mapped_sha256"]
    assert hashlib.sha256(b"".join(sorted(tail))).hexdigest() == g["tail_multiset_sha256"]
