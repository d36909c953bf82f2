# One measured GPU pass: parity tests, smoke, the default bench (with cpu_baseline),
# a rocprofv3 kernel-trace/stats profile of the same bench, and separate PMC passes for HBM bytes.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { tail -30 $OUT/prof_bench.err; exit 1; }
cat $OUT/prof_bench.json
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C -d $OUT/pmc_$C -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-realign > $OUT/pmc_$C.json 2> $OUT/pmc_$C.err || { tail -20 $OUT/pmc_$C.err; exit 1; }
done
echo done
