"""Per-kernel derived metrics from rocprofv3 --pmc runs: python tools/pmc_table.py DIR pass1 pass2 ..."""
import collections
import csv
import sys

d0 = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for p in sys.argv[2:]:
    for r in csv.DictReader(open(f"{d0}/{p}/run_counter_collection.csv")):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:30]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
print(f"{'kernel':30s} {'waves':>8s} {'actv%':>6s} {'wait%':>6s} {'waitI%':>6s} {'valu%':>6s} {'lds%':>6s} {'ldsI/w':>7s} "
      f"{'bankc/ldsI':>10s} {'valuI/w':>8s} {'saluI/w':>8s} {'fetchGB':>8s} {'writeGB':>8s}")
for k, d in sorted(agg.items()):
    wc = d["SQ_WAVE_CYCLES"] or 1
    w = max(d["SQ_WAVES"], 1)
    print(f"{k:30s} {d['SQ_WAVES']:8.3g} {100*d['SQ_ACTIVE_INST_ANY']/wc:6.1f} {100*d['SQ_WAIT_ANY']/wc:6.1f} "
          f"{100*d['SQ_WAIT_INST_ANY']/wc:6.1f} {100*d['SQ_ACTIVE_INST_VALU']/wc:6.1f} {100*d['SQ_ACTIVE_INST_LDS']/wc:6.1f} "
          f"{d['SQ_INSTS_LDS']/w:7.0f} {d['SQ_LDS_BANK_CONFLICT']/max(d['SQ_INSTS_LDS'],1):10.2f} "
          f"{d['SQ_INSTS_VALU']/w:8.0f} {d['SQ_INSTS_SALU']/w:8.0f} {2*d['FETCH_SIZE']*1024/1e9:8.2f} {d['WRITE_SIZE']*1024/1e9:8.2f}")
