"""GPU: inputs larger than HBM (oge_sort_markdup_chunked, csrc/chunked.hip): with chunk sizes forced
tiny (many sorted runs spilled into the host arena, many key ranges cut from them), the output equals
the whole-input one-GPU output (oge_sort_markdup_dev / sort + gather) byte for byte, sort and
sort + dedup, on the reference goldens and synthetic sets (the reference's runs + merge,
alg/read_sorter.cpp:48-190, for any input size)."""
import numpy as np
import pytest

from goldens import CASE_NAMES, load_case
from openge_amd import lib as L
from test_gpu_dist import _single

pytestmark = pytest.mark.gpu


def _check(ctx, recs, offs, n_ref, header, chunk, sort_only=False):
    n = len(offs) - 1
    opts = None if sort_only else L.markdup_opts_from_header(header, n_ref)[0]
    want, nd = _single(ctx, recs, offs, n, n_ref, opts)
    spill = recs.copy()  # the arena becomes the spill space
    got, gd, runs, ranges = L.sort_markdup_chunked(ctx, spill, offs, n, n_ref, opts, chunk)
    assert got == want
    assert gd == nd
    return runs, ranges


@pytest.mark.parametrize("name", CASE_NAMES)
def test_chunked_equals_whole_on_goldens(ctx, name):
    c = load_case(name)
    total = int(c.offs[-1] - c.offs[0])
    chunk = max(1 << 16, total // 7)
    runs, ranges = _check(ctx, c.recs, c.offs, c.n_ref, c.header, chunk)
    if total > 4 * chunk:
        assert runs > 1 and ranges > 1
    _check(ctx, c.recs, c.offs, c.n_ref, c.header, chunk, sort_only=True)


@pytest.mark.parametrize("preset,pairs,seed,parts", [("c2", 60000, 3, 9), ("mix", 8000, 4, 5), ("c2", 20000, 5, 40)])
def test_chunked_equals_whole_synthetic(ctx, preset, pairs, seed, parts):
    p = L.synth_params(pairs, preset=preset, seed=seed)
    recs, offs, hdr = L.synth_host(p)
    total = int(offs[-1] - offs[0])
    runs, ranges = _check(ctx, recs, offs, p.n_ref, hdr, max(1 << 16, total // parts))
    assert runs >= parts - 1 and ranges >= parts - 1


def test_chunked_tie_pile_larger_than_chunk_fails_loudly(ctx):
    import bamutil
    recs = [bamutil.make_record(f"r{i:06d}", 0, 0, 1000, "100M", "A" * 100) for i in range(3000)]
    rr, oo = bamutil.pack_records(recs)
    hdr = "@HD\tVN:1.0\tSO:unsorted\n@SQ\tSN:chr1\tLN:100000\n"
    with pytest.raises(L.OgeError, match="share one sort key"):
        L.sort_markdup_chunked(ctx, rr.copy(), oo, len(oo) - 1, 1, None, 1 << 16)
