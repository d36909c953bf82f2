# parity tests, full bench, kernel profile at 50M reads
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -30 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --pairs 25000000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err || { tail -30 gpurun_out/prof/bench.err; exit 1; }
cut -d, -f1-4 gpurun_out/prof/run_kernel_stats.csv | head -25
