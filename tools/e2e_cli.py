"""End-to-end `openge mergesort -M` BAM -> BAM timing on a C2-shaped synthetic BAM (N reads).

usage: python tools/e2e_cli.py N_READS OUTDIR [threads]
Writes OUTDIR/c2_<N>.bam (BGZF level 6, product writer), runs the CLI, prints one JSON line."""
import json
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from openge_amd import lib as L  # noqa: E402

n = int(sys.argv[1])
out = Path(sys.argv[2])
th = int(sys.argv[3]) if len(sys.argv) > 3 else 16
out.mkdir(parents=True, exist_ok=True)
src = out / f"c2_{n}.bam"
if not src.exists():
    t = time.perf_counter()
    p = L.synth_params(n // 2, preset="c2", seed=1234)
    recs, offs, hdr = L.synth_host(p, threads=th)
    print(f"synth {n} reads in {time.perf_counter() - t:.1f} s", file=sys.stderr, flush=True)
    L.write_bam(src, hdr, recs, offs, n, level=6, threads=th)
    print(f"wrote {src} ({src.stat().st_size / 1e9:.2f} GB) in {time.perf_counter() - t:.1f} s", file=sys.stderr,
          flush=True)
    del recs, offs
import os  # noqa: E402

# E2E_POOL="1,0": one run per setting of OGE_POOL (the CLI's device memory pool), output removed between
for pool in os.environ.get("E2E_POOL", "default").split(","):
    env = dict(os.environ)
    if pool != "default":
        env["OGE_POOL"] = pool
    dst = out / "sorted_dedup.bam"
    if dst.exists():
        dst.unlink()
    t0 = time.perf_counter()
    r = subprocess.run([str(ROOT / "openge_amd/openge"), "mergesort", "-M", "--nopg", "-v", "-t", str(th), str(src), "-o",
                        str(dst)], capture_output=True, text=True, env=env)
    dt = time.perf_counter() - t0
    print(json.dumps({"reads": n, "pool": pool, "seconds": round(dt, 3), "mreads_per_s": round(n / dt / 1e6, 3),
                      "threads": th, "rc": r.returncode, "stderr_tail": r.stderr[-1500:],
                      "in_bytes": src.stat().st_size}), flush=True)
