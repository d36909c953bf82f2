"""Full-size parity pins made by the REFERENCE itself (run in the build container only; minutes).

oracle/_ref/ref_driver (OpenGE's own modules compiled from /root/reference by oracle/Makefile.ref) is run
on config-scale inputs rebuilt at test time from their generator parameters, and its outputs are
reduced to digests (tests/golden/large.json):
  c2_4m   C2 generator (24 GRCh38-shaped contigs, 8% duplicate pairs, 1% inter-contig,
          0.5% mate-unmapped, 2 libraries), 2M pairs = 4M reads, seed 4242:
            sort           -> sha256 of the output record stream, header text
            sortdedup -v   -> the same + number of 0x400 records + sha256 of their output indices
  c5_50k  the C5 local-realignment set (50,000 indel intervals on 24 contigs, 4M reads, the bench's
          default parameters): realign -> sha256 of the output record stream, header text, count
The record streams are hashed exactly as written (decompressed BAM bytes after the header).

Usage:  python tests/golden/make_large_goldens.py
"""
from __future__ import annotations

import gzip
import hashlib
import json
import struct
import subprocess
import sys
import tempfile
import time
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))

import oracle  # noqa: E402
from openge_amd import lib as L  # noqa: E402

C2 = {"preset": "c2", "n_pairs": 2_000_000, "seed": 4242}


def split_bam(raw: bytes):
    """-> (header text, record stream bytes) of a decompressed BAM."""
    (lt,) = struct.unpack_from("<i", raw, 4)
    text = raw[8:8 + lt].decode()
    p = 8 + lt
    (nref,) = struct.unpack_from("<i", raw, p)
    p += 4
    for _ in range(nref):
        (ln,) = struct.unpack_from("<i", raw, p)
        p += 8 + ln
    return text, raw[p:]


def flag_dups(stream: bytes):
    idx, q, k = [], 0, 0
    while q < len(stream):
        (bs,) = struct.unpack_from("<I", stream, q)
        if stream[q + 19] & 0x04:
            idx.append(k)
        q += 4 + bs
        k += 1
    return k, idx


def digest_file(path: Path) -> dict:
    text, stream = split_bam(gzip.decompress(path.read_bytes()))
    n, dups = flag_dups(stream)
    import numpy as np
    return {"header": text, "stream_sha256": hashlib.sha256(stream).hexdigest(), "n": n, "n_dup": len(dups),
            "dup_idx_sha256": hashlib.sha256(np.array(dups, dtype=np.uint32).tobytes()).hexdigest()}


def run(driver, *args, timeout=1800):
    t0 = time.time()
    subprocess.run([str(driver), *map(str, args)], check=True, capture_output=True, timeout=timeout)
    return time.time() - t0


def main():
    driver = oracle.build_ref()
    assert driver and driver.exists(), "reference harness could not be built"
    out = {}
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        tmp = Path(td)
        p = L.synth_params(C2["n_pairs"], preset=C2["preset"], seed=C2["seed"])
        recs, offs, hdr = L.synth_host(p)
        src = tmp / "c2.bam"
        L.write_bam(src, hdr, recs, offs, 2 * C2["n_pairs"], level=1, threads=8)
        del recs, offs
        t_sort = run(driver, "sort", "-t", 8, "-T", tmp, src, tmp / "s.bam")
        t_sd = run(driver, "sortdedup", "-v", "-t", 8, "-T", tmp, src, tmp / "sd.bam")
        out["c2_4m"] = {"spec": C2, "sort": digest_file(tmp / "s.bam"), "sortdedup_v": digest_file(tmp / "sd.bam"),
                        "reference_seconds": {"sort": round(t_sort, 1), "sortdedup": round(t_sd, 1)}}
        print("c2_4m", out["c2_4m"]["sortdedup_v"]["n_dup"], t_sort, t_sd, flush=True)
        rp = L.realign_synth_params()
        fa, iv, bam = L.synth_realign(rp, td, level=1, threads=8)
        t_rl = run(driver, "realign", "-t", 8, "-R", fa, "-L", iv, bam, tmp / "rl.bam")
        d = digest_file(tmp / "rl.bam")
        out["c5_50k"] = {"spec": {k: getattr(rp, k) for k, _ in L.RealignSynthParams._fields_},
                         "realign": {k: d[k] for k in ("header", "stream_sha256", "n")},
                         "reference_seconds": round(t_rl, 1)}
        print("c5_50k", d["n"], t_rl, flush=True)
    (HERE / "large.json").write_text(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
