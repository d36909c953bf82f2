import json, csv, sys
d = json.load(open('gpurun_out/bench_full.json'))
print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'], d['pipeline']['achieved'], d['stages_ms'], d.get('cpu_baseline', {}).get('value'))
rows = list(csv.DictReader(open('gpurun_out/prof/run_kernel_stats.csv')))
for r in rows[:int(sys.argv[1]) if len(sys.argv) > 1 else 14]:
    print(f"{r['Name'][:60]:60s} calls={r['Calls']:>4s} avg_ms={float(r['AverageNs'])/1e6:8.3f} tot_ms={float(r['TotalDurationNs'])/1e6:8.2f}")
