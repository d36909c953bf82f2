# sort primitives + sort/dedup parity on the GPU, then the bench (no realign / cpu legs)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-sort}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_prims.py tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_shard.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-realign > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 - <<'PY' $OUT
import csv, sys, json
d = json.load(open(sys.argv[1] + "/bench.json"))
print(d["value"], d["ms_per_step"], d["stages_ms"], d["roofline"]["frac"])
rows = list(csv.DictReader(open(sys.argv[1] + "/prof/run_kernel_stats.csv")))
for r in rows[:14]:
    print(f"{r['Name'][:60]:60s} calls={r['Calls']:>4s} avg_ms={float(r['AverageNs'])/1e6:8.3f} tot_ms={float(r['TotalDurationNs'])/1e6:9.2f}")
PY
