"""GPU: mergesort's extras through the C ABI and the CLI -- Filter (-r/-q) as a device compaction
(oge_filter_records_dev) and sort by name (-b, oge_sort_name_dev) -- against the REFERENCE's own
outputs (tests/golden/extras) and the oracle on seeded inputs."""
import subprocess

import numpy as np
import pytest
import torch

import bamutil
import oracle
from extras_util import (EXTRA_CASES, canonical_name_digests, check_filtered_perm, load_extras, opts_dict,
                         oracle_filtered_sort, refs_of)
from goldens import GOLDEN
from openge_amd import lib as L

pytestmark = pytest.mark.gpu
OPENGE = str(L.PKG / "openge")


@pytest.fixture(scope="module", params=EXTRA_CASES)
def ex(request, built):
    return load_extras(request.param)


def dev_filter(ctx, recs, offs, n, **kw):
    """-> input indices of the records oge_filter_records_dev keeps (via the output bytes)."""
    d_recs = torch.from_numpy(np.ascontiguousarray(recs)).cuda()
    d_off = torch.from_numpy(np.ascontiguousarray(offs[:n + 1]).view(np.int64)).cuda()
    d_out = torch.zeros(max(int(offs[n]) + 64, 64), dtype=torch.uint8, device="cuda")
    d_oo = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    m = ctx.filter_records_dev(d_recs.data_ptr(), d_off.data_ptr(), n, L.filter_opts(**kw), d_out.data_ptr(),
                               d_oo.data_ptr())
    ctx.sync()
    return d_out.cpu().numpy(), d_oo.cpu().numpy().view(np.uint64)[:m + 1], m


def kept_records_equal(recs, offs, keep, out, oo, m):
    kept = np.nonzero(keep)[0]
    assert m == len(kept)
    assert int(oo[0]) == 0
    for k, i in enumerate(kept):
        a = bamutil.rec_bytes(recs, offs[i])
        b = bamutil.rec_bytes(out, oo[k])
        assert a[:14] == b[:14] and a[16:] == b[16:], k  # bin is recomputed by the gather


def test_filter_dev_matches_oracle_on_goldens(ctx, ex):
    case, meta, _ = ex
    refs = refs_of(case.header)
    for key, g in meta["filters"].items():
        kw = opts_dict(g["opts"], refs)
        out, oo, m = dev_filter(ctx, case.recs, case.offs, case.n, **kw)
        assert m == g["n_out"], key
        kept_records_equal(case.recs, case.offs, oracle.filter_keep(case.recs, case.offs, case.n, **kw), out, oo, m)


@pytest.mark.parametrize("kw", [
    dict(mapq_min=25),
    dict(min_len=120, max_len=149),
    dict(count_limit=777, mapq_min=10),
    dict(count_limit=0),
    dict(has_region=1, ref_id=3, left_pos=1_000_000, right_pos=30_000_000, mapq_min=40),
])
def test_filter_dev_matches_oracle_synthetic(ctx, kw):
    p = L.synth_params(40000, preset="mix", seed=31)
    recs, offs, _ = L.synth_host(p)
    n = 80000
    out, oo, m = dev_filter(ctx, recs, offs, n, **kw)
    keep = oracle.filter_keep(recs, offs, n, **kw)
    kept_records_equal(recs, offs, keep, out, oo, m)


def test_sort_name_matches_oracle_on_goldens(ctx, ex):
    case, meta, _ = ex
    perm = ctx.sort_name(case.recs, case.offs[:-1].copy(), case.n)
    assert np.array_equal(perm, oracle.sort_name_perm(case.recs, case.offs, case.n))
    rbs = [bamutil.rec_bytes(case.recs, case.offs[i]) for i in perm]
    assert canonical_name_digests(rbs) == (meta["byname"]["names_sha256"], meta["byname"]["canonical_sha256"])


def test_sort_name_ragged_names(ctx):
    """Names of 1..40 bytes incl. prefixes of each other, high bytes, many exact ties (input order)."""
    rng = np.random.default_rng(5)
    alpha = np.frombuffer(b"ab\x7f\xfeZ09_", dtype=np.uint8)
    base = [bytes(rng.choice(alpha, size=int(rng.integers(1, 41)))) for _ in range(3000)]
    names = base + [b[:max(1, len(b) // 2)] for b in base[:800]] + [base[i] for i in rng.integers(0, 3000, 2000)]
    order = rng.permutation(len(names))
    recs = [bamutil.make_record(names[i].decode("latin-1"), 0, 0, int(k), "") for k, i in enumerate(order)]
    rr, oo = bamutil.pack_records(recs)
    n = len(recs)
    perm = ctx.sort_name(rr, oo[:-1].copy(), n)
    assert np.array_equal(perm, oracle.sort_name_perm(rr, oo, n))
    got = [bamutil.rec_bytes(rr, oo[i])[36:36 + rr[int(oo[i]) + 12] - 1] for i in perm]
    assert got == sorted(got)


def test_sort_name_empty_and_single(ctx):
    rr, oo = bamutil.pack_records([bamutil.make_record("x", 0, 0, 1, "")])
    assert ctx.sort_name(rr, oo[:-1].copy(), 1).tolist() == [0]
    assert len(ctx.sort_name(rr, oo[:-1].copy(), 0)) == 0


def test_sort_name_synthetic_large(ctx):
    p = L.synth_params(500000, preset="c2", seed=77)
    recs, offs, _ = L.synth_host(p)
    n = 1_000_000
    perm = ctx.sort_name(recs, offs[:-1].copy(), n)
    assert np.array_equal(perm, oracle.sort_name_perm(recs, offs, n))


# ------------------------------------------------------------------------------------------ CLI
def run(*args, ok=True):
    r = subprocess.run([OPENGE, *map(str, args)], capture_output=True, text=True, timeout=300)
    if ok:
        assert r.returncode == 0, r.stderr
    return r


def case_input(case, tmp_path):
    if case.meta["spec"]["kind"] == "file":
        return GOLDEN / "inputs" / case.meta["spec"]["file"]
    path = tmp_path / "in.bam"
    bamutil.write_bam_py(path, case.header, refs_of(case.header), [bamutil.rec_bytes(case.recs, o) for o in case.offs[:-1]])
    return path


def test_cli_mergesort_filters_match_reference(ex, tmp_path):
    case, meta, arrays = ex
    src = case_input(case, tmp_path)
    for key, g in meta["filters"].items():
        dst = tmp_path / f"{key}.bam"
        run("mergesort", "--nopg", *g["opts"], src, "-o", dst)
        h, _, r, o = bamutil.read_bam(dst)
        assert h == g["header"], key
        assert len(o) == g["n_out"], key
        check_filtered_perm(case, bamutil.perm_of(r, o, case.recs, case.offs[:-1]), arrays[f"perm_{key}"])


def test_cli_mergesort_M_with_filter_matches_reference(ex, tmp_path):
    case, meta, arrays = ex
    g = meta["sortdedup"]["r_range_q30"]
    dst = tmp_path / "sd.bam"
    run("mergesort", "-M", "--nopg", *g["opts"], case_input(case, tmp_path), "-o", dst)
    _, _, r, o = bamutil.read_bam(dst)
    assert len(o) == g["n_out"]
    idx = np.nonzero(bamutil.flags_of(r, o) & 0x400)[0].astype(np.uint32)
    assert np.array_equal(idx, arrays["dup_r_range_q30"])


def test_cli_mergesort_byname_matches_reference(ex, tmp_path):
    case, meta, _ = ex
    dst = tmp_path / "bn.bam"
    run("mergesort", "-b", "--nopg", case_input(case, tmp_path), "-o", dst)
    h, _, r, o = bamutil.read_bam(dst)
    assert h == meta["byname"]["header"]
    rbs = [bamutil.rec_bytes(r, x) for x in o]
    assert canonical_name_digests(rbs) == (meta["byname"]["names_sha256"], meta["byname"]["canonical_sha256"])


def test_cli_byname_then_dedup_equals_dedup_of_name_sorted(ex, tmp_path):
    """-b -M: the chain sorts by name, then MarkDuplicates runs over the name-sorted stream."""
    case, _, _ = ex
    src = case_input(case, tmp_path)
    run("mergesort", "-b", "--nopg", src, "-o", tmp_path / "bn.bam")
    run("dedup", "--nopg", tmp_path / "bn.bam", "-o", tmp_path / "bn_d.bam")
    run("mergesort", "-b", "-M", "--nopg", src, "-o", tmp_path / "bn_m.bam")
    a, b = bamutil.read_bam(tmp_path / "bn_d.bam"), bamutil.read_bam(tmp_path / "bn_m.bam")
    assert a[0] == b[0] and np.array_equal(a[2], b[2])


@pytest.mark.parametrize("region,msg", [("nosuchchrom", "Can't find chromosome'nosuchchrom'"),
                                        ("YHet:999999999", "after end of the reference sequence")])
def test_cli_bad_region_fails_like_reference(built, tmp_path, region, msg):
    r = run("mergesort", "--nopg", "-r", region, GOLDEN / "inputs" / "208.yhet.bam", "-o", tmp_path / "x.bam", ok=False)
    assert r.returncode != 0
    assert msg in r.stderr and "could not parse region" in r.stderr


def write_parts(case, order, k, tmp_path, tag):
    refs = refs_of(case.header)
    paths = []
    for f in range(k):
        p = tmp_path / f"{tag}{f}.bam"
        bamutil.write_bam_py(p, case.header, refs, [bamutil.rec_bytes(case.recs, case.offs[i]) for i in order[f::k]])
        paths.append(p)
    return paths


@pytest.mark.parametrize("name", ["yhet208", "mix3k", "c2_20k"])
@pytest.mark.parametrize("tag", ["unsorted", "sorted"])
def test_cli_dedup_multiple_inputs_matches_reference(built, tmp_path, name, tag):
    """openge dedup a.bam b.bam c.bam: MultiReader's interleaving (read_stream_reader.h:132-153)."""
    case, meta, arrays = load_extras(name)
    k = meta["multi"][tag]["k"]
    order = np.arange(case.n) if tag == "unsorted" else oracle.sort_perm(case.recs, case.offs, case.n)
    parts = write_parts(case, order, k, tmp_path, tag)
    dst = tmp_path / "out.bam"
    run("dedup", "--nopg", *parts, "-o", dst)
    h, _, r, o = bamutil.read_bam(dst)
    assert h == meta["multi"][tag]["header"]
    assert np.array_equal(bamutil.perm_of(r, o, case.recs, case.offs[:-1]), arrays[f"multi_{tag}_order"])
    idx = np.nonzero(bamutil.flags_of(r, o) & 0x400)[0].astype(np.uint32)
    assert np.array_equal(idx, arrays[f"multi_{tag}_dup"])


def test_cli_mergesort_multiple_inputs_equals_single(built, tmp_path):
    case, _, _ = load_extras("mix3k")
    parts = write_parts(case, np.arange(case.n), 3, tmp_path, "p")
    src = tmp_path / "whole.bam"
    bamutil.write_bam_py(src, case.header, refs_of(case.header), [bamutil.rec_bytes(case.recs, o) for o in case.offs[:-1]])
    run("mergesort", "-M", "--nopg", *parts, "-o", tmp_path / "a.bam")
    run("mergesort", "-M", "--nopg", src, "-o", tmp_path / "b.bam")
    a, b = bamutil.read_bam(tmp_path / "a.bam"), bamutil.read_bam(tmp_path / "b.bam")
    assert a[0] == b[0]
    ra = [bamutil.rec_bytes(a[2], o) for o in a[3]]
    rb = [bamutil.rec_bytes(b[2], o) for o in b[3]]
    m = sum(int.from_bytes(x[4:8], "little", signed=True) != -1 for x in rb)
    assert ra[:m] == rb[:m]  # the refID -1 tail keeps input order, which differs
    assert sorted(ra[m:]) == sorted(rb[m:])
