"""Per-kernel table from rocprofv3 counter CSVs: average per launch of each counter and the isolated
duration (counter collection serialises kernels).  usage: python tools/pmc_table.py DIR [DIR...]"""
import collections
import csv
import sys
from pathlib import Path

agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(dict)
for d in sys.argv[1:]:
    for f in Path(d).rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k][(f, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for k, cs in agg.items():
    ds = list(dur[k].values())
    print(f"{k}: launches {len(ds) // max(1, len(sys.argv) - 1)}, isolated ms/launch {sum(ds) / len(ds):.3f}")
    for c, v in sorted(cs.items()):
        print(f"    {c:24s} {sum(v) / len(v):.4e}")
