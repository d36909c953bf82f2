"""Summarise a gpurun round directory into profiles/: kernel stats + PMC HBM bytes per kernel.

usage: python tools/pmc_summary.py gpurun_out/<tag> profiles/<tag>

HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes).  With a pmc_SQ_INSTS_VALU pass
also the VALU wave-instructions per launch (bench.py: x 64 lanes / stage time / 78.6 T lane-ops/s).  The factor 2 on FETCH_SIZE is
the gfx950 correction of /opt/skills/guides/MI355X_MICROARCH.md ("HBM" section): FETCH_SIZE counts
64 B per 128 B memory-side read request of a wide (16 B/lane) streaming read.  WRITE_SIZE is exact
for 16 B/lane streaming stores.  FETCH_SIZE and WRITE_SIZE come from separate --pmc passes.
"""
import csv
import json
import shutil
import sys
from pathlib import Path


def per_kernel(path, totals=None, scale=1024.0):
    agg = {}
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        agg.setdefault(k, []).append(float(r["Counter_Value"]) * scale)
    if totals is not None:
        totals.update({k: sum(v) for k, v in agg.items()})
    return {k: sum(v) / len(v) for k, v in agg.items()}


# stages made of several kernels / launches (STAGES="k_defl=2,k_infl=1": the prefix and how many times
# the stage ran in the profiled command): one entry per stage with its bytes per run, listed first so
# bench.py's pmc_traffic finds the stage before any single kernel of it
def stage_entries(ft, wt, spec, vt=None):
    import re
    out = {}
    for item in filter(None, spec.split(",")):
        pre, runs = item.split("=")
        m = re.compile(re.escape(pre) + r"[_(<]").search  # k_infl: k_infl_*; k_infl_huff: that kernel alone
        f = sum(v for k, v in ft.items() if m(k)) / float(runs)
        w = sum(v for k, v in wt.items() if m(k)) / float(runs)
        e = {"fetch_size_bytes": f, "write_size_bytes": w, "hbm_bytes": 2 * f + w}
        if vt:
            e["valu_insts"] = sum(v for k, v in vt.items() if m(k)) / float(runs)
        out[f"{pre} (stage: all {pre}_* launches of one run)"] = e
    return out


def main():
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    dst.parent.mkdir(parents=True, exist_ok=True)
    stats = src / "prof" / "run_kernel_stats.csv"
    if stats.exists():
        shutil.copy(stats, str(dst) + "_kernel_stats.csv")
    for j in ["bench.json", "prof_bench.json"]:
        if (src / j).exists():
            shutil.copy(src / j, str(dst) + "_" + j)
    fetch = src / "pmc_FETCH_SIZE" / "run_counter_collection.csv"
    write = src / "pmc_WRITE_SIZE" / "run_counter_collection.csv"
    if not (fetch.exists() and write.exists()):
        return
    import os
    ft, wt, vt = {}, {}, {}
    f, w = per_kernel(fetch, ft), per_kernel(write, wt)
    valu = src / "pmc_SQ_INSTS_VALU" / "run_counter_collection.csv"
    v = per_kernel(valu, vt, scale=1.0) if valu.exists() else {}
    bench = json.loads((src / "pmc_FETCH_SIZE.json").read_text())
    out = {"workload": bench["config"], "note": "per launch; hbm bytes = 2*FETCH_SIZE + WRITE_SIZE; valu_insts = "
                                                "SQ_INSTS_VALU (wave instructions)",
           "kernels": stage_entries(ft, wt, os.environ.get("STAGES", ""), vt)}
    for k in sorted(set(f) | set(w), key=lambda k: -(2 * f.get(k, 0) + w.get(k, 0))):
        out["kernels"][k] = {"fetch_size_bytes": f.get(k), "write_size_bytes": w.get(k),
                             "hbm_bytes": 2 * f.get(k, 0) + w.get(k, 0)}
        if k in v:
            out["kernels"][k]["valu_insts"] = v[k]
    Path(str(dst) + "_pmc.json").write_text(json.dumps(out, indent=1))
    print(f"wrote {dst}_pmc.json")


if __name__ == "__main__":
    main()
