"""Generate the parity goldens from the REFERENCE itself (run in the build container only).

oracle/_ref/ref_driver is the reference's own ReadSorter / MarkDuplicates modules compiled from
/root/reference (oracle/Makefile.ref).  For every case below it is run as
  sort            (mergesort, no -M)
  dedup -v        on the reference's sorted output and on the unsorted input
  dedup           (non-verbose) on the unsorted input
  sortdedup -v    (mergesort -M --nosplit)
  dedup -v -K k   (split-by-chromosome chains, the reference's default without --nosplit; k = 3, 12)
                  on the sorted output, and sortdedup -v -K 3
and the outputs are reduced to small fixtures: the sort permutation (input index per output
record), indices of records carrying 0x400, SHA-256 digests of the output record streams and the
regenerated header text.  Inputs are either fixtures the reference's own tests hold
(openge/test/data/*.bam, copied into inputs/) or deterministic synthetic sets rebuilt from their
parameters at test time.

Usage:  python tests/golden/make_goldens.py
"""
from __future__ import annotations

import hashlib
import json
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import bamutil  # noqa: E402
import oracle  # noqa: E402
from golden.edge_cases import HEADER as EDGE_HEADER, REFS as EDGE_REFS, build_edge_records  # noqa: E402
from openge_amd import lib as L  # noqa: E402

REF_DATA = Path("/root/reference/openge/test/data")
CASES = {
    "simple": {"kind": "file", "file": "simple.bam"},
    "yhet208": {"kind": "file", "file": "208.yhet.bam"},
    "edge": {"kind": "edge"},
    "mix3k": {"kind": "synth", "preset": "mix", "n_pairs": 3000, "seed": 7},
    "c2_20k": {"kind": "synth", "preset": "c2", "n_pairs": 20000, "seed": 99},
    "c1_100k": {"kind": "synth", "preset": "c1", "n_pairs": 50000, "seed": 1234},
}
FULL_ARRAYS_MAX = 20000
SPLIT_K = (3, 12)


def materialize(name: str, spec: dict, tmp: Path) -> Path:
    """Write the case input as a BAM file and return its path."""
    if spec["kind"] == "file":
        dst = HERE / "inputs" / spec["file"]
        dst.parent.mkdir(exist_ok=True)
        if not dst.exists():
            shutil.copy(REF_DATA / spec["file"], dst)
        return dst
    path = tmp / f"{name}.bam"
    if spec["kind"] == "edge":
        bamutil.write_bam_py(path, EDGE_HEADER, EDGE_REFS, build_edge_records())
        return path
    p = L.synth_params(spec["n_pairs"], preset=spec["preset"], seed=spec["seed"])
    recs, offs, hdr = L.synth_host(p)
    L.write_bam(path, hdr, recs, offs, 2 * spec["n_pairs"])
    return path


def stream_digests(recs, offs) -> dict:
    """sha256 of the mapped record stream in order, and of the refID==-1 tail as a sorted multiset."""
    h = hashlib.sha256()
    tail = []
    for o in offs:
        rb = bamutil.rec_bytes(recs, o)
        if int.from_bytes(rb[4:8], "little", signed=True) == -1:
            tail.append(rb)
        else:
            h.update(rb)
    t = hashlib.sha256(b"".join(sorted(tail)))
    return {"mapped_sha256": h.hexdigest(), "tail_multiset_sha256": t.hexdigest(), "n_tail": len(tail)}


def run(driver, mode, src, dst, *extra):
    subprocess.run([str(driver), mode, *extra, "-T", str(dst.parent), str(src), str(dst)], check=True,
                   capture_output=True, timeout=600)


def main():
    driver = oracle.build_ref()
    assert driver and driver.exists(), "reference harness could not be built"
    with tempfile.TemporaryDirectory() as td:
        tmp = Path(td)
        for name, spec in CASES.items():
            src = materialize(name, spec, tmp)
            out = HERE / name
            out.mkdir(exist_ok=True)
            hdr_in, _, irecs, ioffs = bamutil.read_bam(src)
            n = len(ioffs)
            s_path, dv_path = tmp / f"{name}.sorted.bam", tmp / f"{name}.sorted.dedup.bam"
            di_path, dn_path, sd_path = tmp / f"{name}.dedup_v.bam", tmp / f"{name}.dedup_nv.bam", tmp / f"{name}.sd.bam"
            run(driver, "sort", src, s_path)
            run(driver, "dedup", s_path, dv_path, "-v")
            run(driver, "dedup", src, di_path, "-v")
            run(driver, "dedup", src, dn_path)
            run(driver, "sortdedup", src, sd_path, "-v")
            split_paths = {}
            for k in SPLIT_K:  # the reference's default split-by-chromosome chains
                split_paths[f"dedup_sorted_v_k{k}"] = tmp / f"{name}.sorted.dedup_k{k}.bam"
                run(driver, "dedup", s_path, split_paths[f"dedup_sorted_v_k{k}"], "-v", "-K", str(k))
            split_paths["sortdedup_v_k3"] = tmp / f"{name}.sd_k3.bam"
            run(driver, "sortdedup", src, split_paths["sortdedup_v_k3"], "-v", "-K", "3")
            hs, _, srecs, soffs = bamutil.read_bam(s_path)
            perm = bamutil.perm_of(srecs, soffs, irecs, ioffs)
            meta = {"case": name, "spec": spec, "n": n, "sorted_header": hs, "sort": stream_digests(srecs, soffs),
                    "perm_sha256": hashlib.sha256(perm.tobytes()).hexdigest()}
            arrays = {}
            for key, path in [("dedup_sorted_v", dv_path), ("dedup_input_v", di_path), ("dedup_input_nv", dn_path),
                              ("sortdedup_v", sd_path)] + sorted(split_paths.items()):
                h, _, r, o = bamutil.read_bam(path)
                fl = bamutil.flags_of(r, o)
                idx = np.nonzero(fl & 0x400)[0].astype(np.uint32)
                meta[key] = {"n_dup": int(len(idx)), "dup_idx_sha256": hashlib.sha256(idx.tobytes()).hexdigest(),
                             "header": h, **stream_digests(r, o)}
                arrays[key] = idx
            if n <= FULL_ARRAYS_MAX:
                arrays["perm"] = perm
            np.savez_compressed(out / "arrays.npz", **arrays)
            (out / "meta.json").write_text(json.dumps(meta, indent=1, sort_keys=True))
            print(f"{name}: n={n} dups(sorted,-v)={meta['dedup_sorted_v']['n_dup']} "
                  f"dups(input,nv)={meta['dedup_input_nv']['n_dup']}")


if __name__ == "__main__":
    main()
