"""Goldens for mergesort's extras from the REFERENCE itself (build container only).

oracle/_ref/ref_driver wires the reference's own FileReader -> Filter -> ReadSorter
(-> MarkDuplicates) chain of command_mergesort.cpp:77-117 (compiled from /root/reference by
oracle/Makefile.ref).  Per case it runs
  sort -r REGION / -q MAPQ / both           (mergesort -r/-q)
  sortdedup -v -r REGION -q MAPQ            (mergesort -M --nosplit -r/-q)
  sort -b                                   (mergesort -b, one temp run)
  dedup -v part0 part1 part2                (several inputs through MultiReader; unsorted and
                                             sorted parts)
and stores: for the filtered sorts the input index of every output record (perm) and digests of
the output record stream; for dedup the 0x400 indices; for -b the output name sequence and a digest
of the output with every run of equal names canonicalised (records sorted bytewise), since the
reference's std::sort leaves the order inside such a run implementation-defined.

Usage:  python tests/golden/make_extras_goldens.py
"""
from __future__ import annotations

import hashlib
import json
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(HERE))

import bamutil  # noqa: E402
import oracle  # noqa: E402
from make_goldens import CASES, materialize, stream_digests  # noqa: E402

OUT = HERE / "extras"
EXTRA_CASES = ["simple", "yhet208", "edge", "mix3k", "c2_20k"]


def filter_sets(refs):
    """Option sets per case, built from its sequence dictionary."""
    (n0, l0) = refs[0]
    (n1, l1) = refs[1] if len(refs) > 1 else refs[0]
    return {
        "q20": ["-q", "20"],
        "q60": ["-q", "60"],
        "r_whole": ["-r", n0],
        "r_range": ["-r", f"{n0}:{l0 // 4}..{l0 // 2}"],
        "r_point": ["-r", f"{n1}:{l1 // 3}"],
        "r_point0": ["-r", f"{n0}:{l0 // 3}"],
        "r_dash": ["-r", f"{n0}:{l0 // 5}-{l0 // 2}"],  # atoi reads "a-b" as the single position a
        "r_range_q30": ["-r", f"{n1}:{l1 // 8}..{(7 * l1) // 8}", "-q", "30"],
    }


def name_of(rb: bytes) -> bytes:
    return rb[36:36 + rb[12] - 1]


def canonical_name_stream(recs, offs) -> tuple[str, str]:
    """(sha of the name sequence, sha of the stream with equal-name runs sorted bytewise, bin field zeroed)."""
    rbs = [bamutil.rec_bytes(recs, o) for o in offs]
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


def run(driver, mode, src, dst, *extra):
    srcs = [str(x) for x in src] if isinstance(src, (list, tuple)) else [str(src)]
    r = subprocess.run([str(driver), mode, *extra, "-T", str(dst.parent), *srcs, str(dst)], capture_output=True,
                       timeout=600)
    return r.returncode


MULTI_CASES = ["yhet208", "mix3k", "c2_20k"]
MULTI_K = 3


def split_inputs(tmp: Path, tag: str, header: str, refs, recs, offs, order) -> list[Path]:
    """Records order[j] for j % K == k go to file k (each file keeps the order given)."""
    paths = []
    for k in range(MULTI_K):
        path = tmp / f"{tag}.part{k}.bam"
        bamutil.write_bam_py(path, header, refs, [bamutil.rec_bytes(recs, offs[i]) for i in order[k::MULTI_K]])
        paths.append(path)
    return paths


def multi_goldens(driver, tmp: Path, name: str, src: Path, meta: dict, arrays: dict) -> None:
    """MultiReader (util/read_stream_reader.h:132-153): dedup -v over K parts of the unsorted input and
    over K parts of the reference-sorted input; output order (input index) and 0x400 indices."""
    hdr, refs, irecs, ioffs = bamutil.read_bam(src)
    s_path = tmp / f"{name}.msorted.bam"
    assert run(driver, "sort", src, s_path) == 0
    _, _, srecs, soffs = bamutil.read_bam(s_path)
    sorted_order = bamutil.perm_of(srecs, soffs, irecs, ioffs)
    meta["multi"] = {}
    for tag, order in (("unsorted", np.arange(len(ioffs))), ("sorted", sorted_order)):
        parts = split_inputs(tmp, f"{name}.{tag}", hdr, refs, irecs, ioffs, order)
        dst = tmp / f"{name}.{tag}.multi.bam"
        assert run(driver, "dedup", parts, dst, "-v") == 0
        h, _, r, o = bamutil.read_bam(dst)
        arrays[f"multi_{tag}_order"] = bamutil.perm_of(r, o, irecs, ioffs)
        idx = np.nonzero(bamutil.flags_of(r, o) & 0x400)[0].astype(np.uint32)
        arrays[f"multi_{tag}_dup"] = idx
        meta["multi"][tag] = {"k": MULTI_K, "n_out": len(o), "n_dup": int(len(idx)), "header": h}


def main():
    driver = oracle.build_ref()
    assert driver and driver.exists(), "reference harness could not be built"
    OUT.mkdir(exist_ok=True)
    with tempfile.TemporaryDirectory() as td:
        tmp = Path(td)
        for name in EXTRA_CASES:
            src = materialize(name, CASES[name], tmp)
            _, refs, irecs, ioffs = bamutil.read_bam(src)
            meta = {"case": name, "n": len(ioffs), "filters": {}, "sortdedup": {}}
            arrays = {}
            for key, opts in filter_sets(refs).items():
                dst = tmp / f"{name}.{key}.bam"
                rc = run(driver, "sort", src, dst, *opts)
                assert rc == 0, (name, key, rc)
                h, _, r, o = bamutil.read_bam(dst)
                perm = bamutil.perm_of(r, o, irecs, ioffs)
                arrays[f"perm_{key}"] = perm
                meta["filters"][key] = {"opts": opts, "n_out": len(o), "header": h, **stream_digests(r, o)}
            opts = filter_sets(refs)["r_range_q30"]
            dst = tmp / f"{name}.sd.bam"
            assert run(driver, "sortdedup", src, dst, "-v", *opts) == 0
            h, _, r, o = bamutil.read_bam(dst)
            idx = np.nonzero(bamutil.flags_of(r, o) & 0x400)[0].astype(np.uint32)
            arrays["dup_r_range_q30"] = idx
            meta["sortdedup"]["r_range_q30"] = {"opts": opts, "n_out": len(o), "n_dup": int(len(idx)),
                                                **stream_digests(r, o)}
            dst = tmp / f"{name}.byname.bam"
            assert run(driver, "sort", src, dst, "-b") == 0
            h, _, r, o = bamutil.read_bam(dst)
            hn, hc = canonical_name_stream(r, o)
            meta["byname"] = {"n_out": len(o), "header": h, "names_sha256": hn, "canonical_sha256": hc}
            if name in MULTI_CASES:
                multi_goldens(driver, tmp, name, src, meta, arrays)
            np.savez_compressed(OUT / f"{name}.npz", **arrays)
            (OUT / f"{name}.json").write_text(json.dumps(meta, indent=1, sort_keys=True))
            print(name, {k: v["n_out"] for k, v in meta["filters"].items()}, "dups", meta["sortdedup"]["r_range_q30"]["n_dup"])


if __name__ == "__main__":
    main()
