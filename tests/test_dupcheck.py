"""CPU: the torch restatement of MarkDuplicates (tests/dupcheck.py), which checks the 300M-read dup set on
the GPU (test_gpu_large.py::test_300m_read_properties), is itself pinned to the REFERENCE's dup sets on
every golden case (tests/golden/*/arrays.npz sortdedup_v, made by oracle/_ref): the cases' records in
ByPosition order (the oracle's permutation) -> the restated 0x400 bits -> the flagged stream positions."""
import numpy as np
import pytest
import torch

import dupcheck
import oracle
from goldens import CASE_NAMES, final_dup_indices, load_case


def _sorted_stream(case):
    perm = oracle.sort_perm(case.recs, case.offs, case.n)
    sizes = np.diff(case.offs.astype(np.int64))[perm]
    off = np.zeros(case.n + 1, np.int64)
    np.cumsum(sizes, out=off[1:])
    buf = np.concatenate([case.recs[int(case.offs[i]):int(case.offs[i + 1])] for i in perm] + [np.zeros(64, np.uint8)])
    return buf, off, perm


@pytest.mark.parametrize("name", CASE_NAMES)
def test_restated_dups_equal_reference(built, name):
    case = load_case(name)
    buf, off, perm = _sorted_stream(case)
    primary, dup = dupcheck.expected_dups(torch.from_numpy(buf), torch.from_numpy(off[:-1]), case.header)
    dup = dup.numpy()
    # {0,1,2} as the goldens' helper takes it: 2 = non-primary (keeps its input bit)
    code = np.where(primary.numpy(), dup.astype(np.uint8), 2).astype(np.uint8)
    sorted_offs = case.offs[perm]
    idx = final_dup_indices(case, sorted_offs, code)
    g = case.meta["sortdedup_v"]
    assert len(idx) == g["n_dup"], (name, len(idx), g["n_dup"])
    assert np.array_equal(idx, case.arrays["sortdedup_v"])


@pytest.mark.parametrize("name", ["c1_100k", "c2_20k"])
def test_restated_mate_join_pairs_equal_names(built, name):
    """Every pair the restatement forms joins two ends of ONE name (consecutive-digit names: r05 found the
    XOR of two name hashes colliding on names that differ in their last digit, at 300M)."""
    case = load_case(name)
    buf, off, perm = _sorted_stream(case)
    dbg = {}
    dupcheck.expected_dups(torch.from_numpy(buf), torch.from_numpy(off[:-1]), case.header, debug=dbg)
    r1, r2 = dbg["pr1"].numpy(), dbg["pr2"].numpy()
    assert len(r1) > 1000

    def nm(i):
        o = int(off[i])
        return bytes(buf[o + 36:o + 36 + int(buf[o + 12]) - 1])

    assert all(nm(a) == nm(b) for a, b in zip(r1, r2))
