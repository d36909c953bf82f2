"""Load the reference-generated golden cases (tests/golden/*) and rebuild their inputs."""
from __future__ import annotations

import hashlib
import json
from dataclasses import dataclass
from pathlib import Path

import numpy as np

import bamutil
from golden.edge_cases import HEADER as EDGE_HEADER, build_edge_records

GOLDEN = Path(__file__).resolve().parent / "golden"
CASE_NAMES = ["simple", "yhet208", "edge", "mix3k", "c2_20k", "c1_100k"]


@dataclass
class Case:
    name: str
    meta: dict
    arrays: dict
    header: str         # input header text as stored
    recs: np.ndarray
    offs: np.ndarray    # n+1 entries
    n: int
    n_ref: int


def load_case(name: str) -> Case:
    meta = json.loads((GOLDEN / name / "meta.json").read_text())
    arrays = dict(np.load(GOLDEN / name / "arrays.npz"))
    spec = meta["spec"]
    if spec["kind"] == "file":
        header, refs, recs, offs = bamutil.read_bam(GOLDEN / "inputs" / spec["file"])
        n_ref = len(refs)
        recs = np.concatenate([recs, np.zeros(16, np.uint8)])
        offs = np.append(offs, np.uint64(len(recs) - 16))
    elif spec["kind"] == "edge":
        header = EDGE_HEADER
        recs, offs = bamutil.pack_records(build_edge_records())
        n_ref = 2
    else:
        from openge_amd import lib as L
        p = L.synth_params(spec["n_pairs"], preset=spec["preset"], seed=spec["seed"])
        recs, offs, header = L.synth_host(p)
        n_ref = p.n_ref
    n = len(offs) - 1
    assert n == meta["n"], (name, n, meta["n"])
    return Case(name, meta, arrays, header, recs, offs, n, n_ref)


def n_mapped_prefix(case: Case, perm: np.ndarray) -> int:
    """Number of leading sorted records with refID != -1."""
    ref = np.array([int.from_bytes(case.recs[int(case.offs[i]) + 4:int(case.offs[i]) + 8].tobytes(), "little",
                                   signed=True) for i in perm])
    return int(np.count_nonzero(ref != -1))


def check_perm(case: Case, perm: np.ndarray) -> None:
    """Exact order for refID >= 0; the refID == -1 tail is implementation-defined."""
    m = n_mapped_prefix(case, perm)
    assert case.n - m == case.meta["sort"]["n_tail"]
    if "perm" in case.arrays:
        g = case.arrays["perm"]
        assert np.array_equal(perm[:m], g[:m])
        assert set(perm[m:].tolist()) == set(g[m:].tolist())
    else:
        assert m == case.n
        assert hashlib.sha256(perm.astype(np.uint32).tobytes()).hexdigest() == case.meta["perm_sha256"]


def final_dup_indices(case: Case, stream_offs: np.ndarray, dup: np.ndarray) -> np.ndarray:
    """Stream positions whose output FLAG carries 0x400: dup==1, or a non-primary record (dup==2)
    that already had 0x400 set (MarkDuplicates leaves non-primary flags alone, :448-453)."""
    pre = np.array([case.recs[int(o) + 19] & 0x04 for o in stream_offs[:case.n]], dtype=np.uint8)
    return np.nonzero((dup == 1) | ((dup == 2) & (pre != 0)))[0].astype(np.uint32)


def check_dups(case: Case, key: str, dup: np.ndarray, stream_offs: np.ndarray) -> None:
    idx = final_dup_indices(case, stream_offs, dup)
    g = case.meta[key]
    assert len(idx) == g["n_dup"], (case.name, key, len(idx), g["n_dup"])
    assert np.array_equal(idx, case.arrays[key])
