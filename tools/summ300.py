import csv, json, sys
d = json.load(open('gpurun_out/prof300/bench.json'))
print(d['value'], d['ms_per_step'], d['stages_ms'])
rows = list(csv.DictReader(open('gpurun_out/prof300/run_kernel_stats.csv')))
for r in rows[:int(sys.argv[1]) if len(sys.argv) > 1 else 30]:
    print(f"{r['Name'][:64]:64s} calls={r['Calls']:>4s} avg_ms={float(r['AverageNs'])/1e6:8.3f} tot_ms={float(r['TotalDurationNs'])/1e6:8.2f}")
