# perf iteration: GPU parity tests for sort/dedup, then the bench under rocprofv3 kernel-trace
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-perf}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_shard.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-realign > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
python3 - <<'PY' $OUT
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1] + "/prof/run_kernel_stats.csv")))
for r in rows[:16]:
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>4s} avg_ms={float(r['AverageNs'])/1e6:8.3f}")
PY
