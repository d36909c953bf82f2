"""The C5 50k realignment pin, made tie-aware from the REFERENCE's own runs (build container only; ~8 min).

The reference picks among consensuses of equal mismatch sum by `random_shuffle` over a
`set<Consensus *>` (alg/local_realignment.cpp:693,711-713): the first of the tied ones in
the shuffled order wins (:764, strictly smaller only), so its output at such an interval is any one of
the tied choices.  Seven plain runs of `ref_driver realign -t 8` on the C5 set gave three different
record streams.  This script runs the reference RUNS times (plain, -t 1, and seeded: `-S s` calls
srand(s) before the chain, so every tied interval gets a fresh shuffle), finds the record windows where
any two runs disagree, and stores in tests/golden/large.json["c5_50k"]["realign"]:

  stable_sha256   sha256 over every record outside the windows, concatenated in order (all runs agree)
  windows         [{lo, hi, variants: [sha256 of records lo..hi as each run wrote them]}]

test_gpu_large.py::test_c5_50k_realign_matches_reference then requires the product's stream to equal
the reference outside the windows and to be one of the reference's variants inside each.

Usage:  python tests/golden/make_c5_variants.py
"""
from __future__ import annotations

import gzip
import hashlib
import json
import sys
import tempfile
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(HERE))

import oracle  # noqa: E402
from openge_amd import lib as L  # noqa: E402
from make_large_goldens import run, split_bam  # noqa: E402

# (threads, seed or None): plain runs keep the reference's own unseeded rand()
RUNS = [(8, None)] * 4 + [(1, None)] + [(8, s) for s in range(11, 21)]
GAP = 2000  # records: disagreements closer than this share one window


def records(stream: bytes):
    out, q = [], 0
    while q < len(stream):
        bs = int.from_bytes(stream[q:q + 4], "little")
        out.append(stream[q:q + 4 + bs])
        q += 4 + bs
    return out


def main():
    driver = oracle.build_ref()
    assert driver and driver.exists(), "reference harness could not be built"
    g = json.loads((HERE / "large.json").read_text())
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        rp = L.realign_synth_params()
        fa, iv, bam = L.synth_realign(rp, td, level=1, threads=8)
        streams = []
        for k, (t, s) in enumerate(RUNS):
            o = Path(td) / f"rl{k}.bam"
            run(driver, "realign", "-t", t, *(["-S", s] if s is not None else []), "-R", fa, "-L", iv, bam, o)
            text, stream = split_bam(gzip.decompress(o.read_bytes()))
            streams.append(records(stream))
            o.unlink()
            print("run", k, t, s, len(streams[-1]), flush=True)
    n = len(streams[0])
    assert all(len(s) == n for s in streams)
    diff = [i for i in range(n) if any(s[i] != streams[0][i] for s in streams[1:])]
    wins = []
    for i in diff:
        if wins and i - wins[-1][1] < GAP:
            wins[-1][1] = i
        else:
            wins.append([i, i])
    inside = set()
    for lo, hi in wins:
        inside.update(range(lo, hi + 1))
    h = hashlib.sha256()
    for i in range(n):
        if i not in inside:
            h.update(streams[0][i])
    windows = []
    for lo, hi in wins:
        vs = sorted({hashlib.sha256(b"".join(s[lo:hi + 1])).hexdigest() for s in streams})
        windows.append({"lo": lo, "hi": hi, "variants": vs})
    rl = g["c5_50k"]["realign"]
    rl.pop("stream_sha256", None)
    rl.update({"n": n, "header": text, "stable_sha256": h.hexdigest(), "windows": windows,
               "reference_runs": [{"threads": t, "seed": s} for t, s in RUNS]})
    (HERE / "large.json").write_text(json.dumps(g, indent=1, sort_keys=True))
    print("windows", [(w["lo"], w["hi"], len(w["variants"])) for w in windows])


if __name__ == "__main__":
    main()
