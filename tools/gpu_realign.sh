# realign GPU pass: realign parity tests, then a bench run with only the realign leg measured in full
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-rl01}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_realign.py -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_rl.log 2>&1 || { tail -40 $OUT/pytest_rl.log; exit 1; }
tail -3 $OUT/pytest_rl.log
timeout -k 10 900 python bench.py --pairs 5000000 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_rl.json 2> $OUT/bench_rl.err || { tail -30 $OUT/bench_rl.err; exit 1; }
cat $OUT/bench_rl.json
