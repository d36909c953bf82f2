"""Shared helpers for the mergesort-extras parity tests (Filter -r/-q, sort by name -b) against the
reference-made goldens in tests/golden/extras (tests/golden/make_extras_goldens.py)."""
from __future__ import annotations

import hashlib
import json

import numpy as np

import oracle
from goldens import GOLDEN, load_case

EXTRAS = GOLDEN / "extras"
EXTRA_CASES = ["simple", "yhet208", "edge", "mix3k", "c2_20k"]


def load_extras(name: str):
    meta = json.loads((EXTRAS / f"{name}.json").read_text())
    arrays = dict(np.load(EXTRAS / f"{name}.npz"))
    return load_case(name), meta, arrays


def refs_of(header: str) -> list[tuple[str, int]]:
    out = []
    for line in header.splitlines():
        if line.startswith("@SQ"):
            f = dict(x.split(":", 1) for x in line.split("\t")[1:])
            out.append((f["SN"], int(f["LN"])))
    return out


def opts_dict(opts: list[str], refs) -> dict:
    """mergesort -r/-q option list -> oracle.filter_keep keywords."""
    d = {}
    it = iter(opts)
    for a in it:
        v = next(it)
        if a == "-q":
            d["mapq_min"] = int(v)
        elif a == "-r":
            r = oracle.parse_region(v, refs)
            assert r is not None, v
            d.update(r)
    return d


def rec_ref(recs, off) -> int:
    return int.from_bytes(recs[int(off) + 4:int(off) + 8].tobytes(), "little", signed=True)


def check_filtered_perm(case, perm: np.ndarray, golden: np.ndarray) -> None:
    """Exact order for refID >= 0; the refID == -1 tail as a set."""
    assert len(perm) == len(golden)
    m = sum(rec_ref(case.recs, case.offs[i]) != -1 for i in perm)
    assert np.array_equal(perm[:m], golden[:m])
    assert set(perm[m:].tolist()) == set(golden[m:].tolist())


def oracle_filtered_sort(case, keep: np.ndarray) -> np.ndarray:
    """Input indices of the kept records in ByPosition order."""
    kept = np.nonzero(keep)[0].astype(np.uint32)
    p = oracle.sort_perm(case.recs, case.offs[:-1][kept], len(kept))
    return kept[p]


def name_of(rb: bytes) -> bytes:
    return rb[36:36 + rb[12] - 1]


def canonical_name_digests(rbs: list[bytes]) -> tuple[str, str]:
    """(sha of the name sequence, sha of the stream with equal-name runs sorted bytewise, bin field zeroed), as
    make_extras_goldens.canonical_name_stream."""
    names = [name_of(rb) for rb in rbs]
    hn = hashlib.sha256(b"\n".join(names)).hexdigest()
    h = hashlib.sha256()
    i = 0
    while i < len(rbs):
        j = i
        while j < len(rbs) and names[j] == names[i]:
            j += 1
        for rb in sorted(rb[:14] + b"\0\0" + rb[16:] for rb in rbs[i:j]):  # bin masked (the writer recomputes it)
            h.update(rb)
        i = j
    return hn, h.hexdigest()
