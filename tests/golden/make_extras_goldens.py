"""Goldens for mergesort's extras from the REFERENCE itself (build container only).

oracle/_ref/ref_driver wires the reference's own FileReader -> Filter -> ReadSorter
(-> MarkDuplicates) chain of command_mergesort.cpp:77-117 (compiled from /root/reference by
oracle/Makefile.ref).  Per case it runs
  sort -r REGION / -q MAPQ / both           (mergesort -r/-q)
  sortdedup -v -r REGION -q MAPQ            (mergesort -M --nosplit -r/-q)
  sort -b                                   (mergesort -b, one temp run)
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
    r = subprocess.run([str(driver), mode, *extra, "-T", str(dst.parent), str(src), str(dst)], capture_output=True,
                       timeout=600)
    return r.returncode


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
            np.savez_compressed(OUT / f"{name}.npz", **arrays)
            (OUT / f"{name}.json").write_text(json.dumps(meta, indent=1, sort_keys=True))
            print(name, {k: v["n_out"] for k, v in meta["filters"].items()}, "dups", meta["sortdedup"]["r_range_q30"]["n_dup"])


if __name__ == "__main__":
    main()
