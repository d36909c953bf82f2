"""Profiling aid: where the `openge localrealign` command's wall time goes on the C5 set -- the CLI with -v
(phase lines with timestamps), a bare process start (`openge version`), and the BAM read alone."""
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from openge_amd import lib as L  # noqa: E402

exe = Path(__file__).resolve().parents[1] / "openge_amd" / "openge"
with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
    p = L.realign_synth_params(n_intervals=50_000)
    fa, iv, bam = L.synth_realign(p, td, level=1, threads=16)
    print("input bam bytes", os.path.getsize(bam), flush=True)
    runs = [({}, ["version"]), ({}, ["localrealign", "--nopg", "-t", "16", "-R", fa, "-L", iv, bam, "-o", os.path.join(td, "o.bam")])]
    for env in ({}, {"OGE_WRITE_DEVICE": "1"}):
        runs.append((dict(env, OGE_WRITE_TRACE="1"), ["localrealign", "-v", "--nopg", "-t", "16", "-R", fa, "-L", iv, bam, "-o",
                                                      os.path.join(td, "o2.bam")]))
    for env, args in runs:
        print("env", env, flush=True)
        t0 = time.perf_counter()
        pr = subprocess.Popen([str(exe)] + args, stderr=subprocess.PIPE, text=True, env=dict(os.environ, **env))
        for line in pr.stderr:
            print(f"  [{time.perf_counter() - t0:7.3f}] {line.rstrip()}", flush=True)
        pr.wait()
        print(args[0], "-v" if "-v" in args else "", "rc", pr.returncode, f"{time.perf_counter() - t0:.3f} s", flush=True)
    print("output bam bytes", os.path.getsize(os.path.join(td, "o.bam")), flush=True)
