"""Host-phase timing of the realign leg on THIS machine's CPU (no GPU): the C5 set (bench.py's realign
leg: 50k intervals, 24 contigs, ~4M reads) through the product's host phases with the oracle scan from
the test harness (tests/native/realign_cpu.cpp).  The scan's results are cached in DIR/scan.bin
(OGE_TEST_SCAN_CACHE), so only the first run pays for the literal scan.

    python tools/realign_prof.py DIR [threads=8] [runs=2] [n_intervals=50000]
"""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import numpy as np  # noqa: E402

from openge_amd import lib as L  # noqa: E402
import realign_util as R  # noqa: E402

d = Path(sys.argv[1])
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 8
runs = int(sys.argv[3]) if len(sys.argv) > 3 else 2
n_iv = int(sys.argv[4]) if len(sys.argv) > 4 else 50_000
d.mkdir(parents=True, exist_ok=True)
fa, iv, bam = str(d / "ref.fa"), str(d / "targets.intervals"), str(d / "reads.bam")
if not Path(bam).exists():
    L.synth_realign(L.realign_synth_params(n_intervals=n_iv), d, level=1, threads=threads)
b = L.Bam(bam, threads=threads)
offs = np.append(b.offs, np.uint64(b.recs.size))
os.environ["OGE_TEST_SCAN_CACHE"] = str(d / "scan.bin")
for r in range(runs):
    st = {}
    t0 = time.perf_counter()
    out, oo = R.realign_cpu(b.header_text, b.recs, offs, b.n, fa, iv, threads=threads, stats=st)
    dt = time.perf_counter() - t0
    print(json.dumps({"run": r, "seconds": round(dt, 3), "reads": b.n, **st}), flush=True)
