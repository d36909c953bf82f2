"""Device inflate throughput by input compressor: the same C2 records (N reads) compressed by the
library's GPU deflate (level 6) and by host libdeflate level 6 (oge_bam_write, the writer samtools-era
tools use), each inflated on the device 3 times (HIP-event stage times).

    python tools/infl_src_ab.py [reads=20000000]"""
import json
import os
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

from openge_amd import lib as L  # noqa: E402

reads = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
p = L.synth_params(reads // 2, preset="c2", seed=1234)
recs, offs, hdr = L.synth_host(p, threads=16)
n = len(offs) - 1
ctx = L.Context(0)
res = {"reads": n}
with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
    path = os.path.join(td, "ld6.bam")
    L.write_bam(path, hdr, recs, offs, n, level=6, threads=16)
    zl = open(path, "rb").read()
payload = recs[: int(offs[-1])].tobytes()
zg = ctx.bgzf_deflate(payload, 6)
for name, z in (("gpu_deflate6", zg), ("libdeflate6", zl)):
    ms = []
    for _ in range(3):
        out = ctx.bgzf_inflate(z)
        ms.append(round(ctx.timing("bgzf_inflate"), 2))
    res[name] = {"compressed": len(z), "out": len(out), "inflate_ms": ms, "GBps": round(len(out) / min(ms) / 1e6, 1)}
    print(name, res[name], file=sys.stderr, flush=True)
print(json.dumps(res))
