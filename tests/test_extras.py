"""CPU: the oracle's restatement of mergesort's extras -- Filter (-r region / -q mapq,
algorithms/filter.cpp:31-249) and sort by name (-b, util/bamtools/Sort.h:67-90) -- pinned to the
REFERENCE's own outputs (tests/golden/extras, made by oracle/_ref from the reference's modules), and
the C ABI's host-side region parser (oge_parse_region) against the same rules."""
import numpy as np
import pytest

import bamutil
import oracle
from extras_util import (EXTRA_CASES, canonical_name_digests, check_filtered_perm, load_extras, opts_dict,
                         oracle_filtered_sort, refs_of)
from goldens import final_dup_indices
from openge_amd import lib as L


@pytest.fixture(scope="module", params=EXTRA_CASES)
def ex(request, built):
    return load_extras(request.param)


def test_oracle_filter_sort_matches_reference(ex):
    case, meta, arrays = ex
    refs = refs_of(case.header)
    for key, g in meta["filters"].items():
        keep = oracle.filter_keep(case.recs, case.offs, case.n, **opts_dict(g["opts"], refs))
        assert int(keep.sum()) == g["n_out"], key
        check_filtered_perm(case, oracle_filtered_sort(case, keep), arrays[f"perm_{key}"])


def test_oracle_filter_sortdedup_matches_reference(ex):
    case, meta, arrays = ex
    g = meta["sortdedup"]["r_range_q30"]
    keep = oracle.filter_keep(case.recs, case.offs, case.n, **opts_dict(g["opts"], refs_of(case.header)))
    order = oracle_filtered_sort(case, keep)
    so = case.offs[:-1][order]
    dup, _ = oracle.markdup(case.recs, so, len(order), case.header)
    assert len(order) == g["n_out"]
    assert np.array_equal(final_dup_indices(case, so, dup), arrays["dup_r_range_q30"])


def test_oracle_sort_name_matches_reference(ex):
    case, meta, _ = ex
    perm = oracle.sort_name_perm(case.recs, case.offs, case.n)
    rbs = [bamutil.rec_bytes(case.recs, case.offs[i]) for i in perm]
    hn, hc = canonical_name_digests(rbs)
    assert hn == meta["byname"]["names_sha256"]
    assert hc == meta["byname"]["canonical_sha256"]


def test_byname_header_says_queryname(ex):
    _, meta, _ = ex
    assert "SO:queryname" in meta["byname"]["header"].splitlines()[0]


def test_parse_region_c_abi_matches_restatement(ex):
    case, meta, _ = ex
    refs = refs_of(case.header)
    for g in meta["filters"].values():
        if "-r" not in g["opts"]:
            continue
        region = g["opts"][g["opts"].index("-r") + 1]
        want = oracle.parse_region(region, refs)
        o = L.parse_region(region, refs)
        assert (o.has_region, o.ref_id, o.left_pos, o.right_pos) == (1, want["ref_id"], want["left_pos"],
                                                                       want["right_pos"])


REFS = [("chrA", 1000), ("chrB", 500), ("chrA", 2000)]


@pytest.mark.parametrize("region,want", [
    ("chrB", (1, 0, 500)),
    ("chrB:10", (1, 10, 10)),
    ("chrB:10..20", (1, 10, 20)),
    ("chrB:10-20", (1, 10, 10)),        # atoi stops at '-' (filter.cpp:76)
    ("chrB:10..", (1, 10, 0)),          # atoi("") = 0
    ("chrB:..20", (1, 0, 20)),
    ("chrA:5..1999", (2, 5, 1999)),     # the last dictionary entry of that name wins (:112-115)
    ("chrB:499..500", (1, 499, 500)),
])
def test_parse_region_forms(built, region, want):
    o = L.parse_region(region, REFS)
    assert (o.ref_id, o.left_pos, o.right_pos) == want
    w = oracle.parse_region(region, REFS)
    assert (w["ref_id"], w["left_pos"], w["right_pos"]) == want


@pytest.mark.parametrize("region,msg", [
    ("", "could not parse"),
    ("chrC", "Can't find chromosome'chrC'"),
    ("chrB:500", "Start position (500) after end of the reference sequence (500)"),
    ("chrB:1..501", "Start position (501) after end of the reference sequence (500)"),
    ("chrB:1..5:9", "could not parse"),
])
def test_parse_region_errors(built, region, msg):
    with pytest.raises(L.OgeError, match=None) as e:
        L.parse_region(region, REFS)
    assert msg in str(e.value)
    assert oracle.parse_region(region, REFS) is None


def test_filter_opts_defaults(built):
    o = L.filter_opts()
    assert (o.has_region, o.mapq_min, o.min_len, o.max_len, o.trim_total, o.count_limit) == (0, 0, 0, 2**31 - 1, 0,
                                                                                             2**31 - 1)


def test_oracle_filter_drops_empty_seq_and_honours_limits(built):
    recs = [bamutil.make_record(f"r{i}", 0, 0, 100 + i, "10M" if i % 3 else "", "ACGTACGTAC" if i % 3 else "",
                                mapq=i % 70) for i in range(60)]
    rr, oo = bamutil.pack_records(recs)
    keep = oracle.filter_keep(rr, oo, 60)
    assert keep.tolist() == [bool(i % 3) for i in range(60)]  # len > trim total (0): empty SEQ is dropped
    keep = oracle.filter_keep(rr, oo, 60, mapq_min=30, count_limit=5)
    want = [i for i in range(60) if i % 3 and i % 70 >= 30][:5]
    assert np.nonzero(keep)[0].tolist() == want


MULTI = ["yhet208", "mix3k", "c2_20k"]


@pytest.mark.parametrize("name", MULTI)
@pytest.mark.parametrize("tag", ["unsorted", "sorted"])
def test_oracle_multireader_dedup_matches_reference(built, name, tag):
    """dedup -v over 3 input files: MultiReader's interleaving, then MarkDuplicates on that stream."""
    case, meta, arrays = load_extras(name)
    g = meta["multi"][tag]
    k = g["k"]
    if tag == "unsorted":
        order = np.arange(case.n)
    else:
        order = oracle.sort_perm(case.recs, case.offs, case.n)
    parts = [order[f::k] for f in range(k)]
    merged = oracle.multireader_order(case.recs, [case.offs[:-1][p] for p in parts])
    out = np.array([parts[f][i] for f, i in merged], dtype=np.uint32)
    assert np.array_equal(out, arrays[f"multi_{tag}_order"])
    so = case.offs[:-1][out]
    dup, _ = oracle.markdup(case.recs, so, case.n, case.header)
    assert np.array_equal(final_dup_indices(case, so, dup), arrays[f"multi_{tag}_dup"])
