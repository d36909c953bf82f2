# iteration loop: GPU parity tests, then a 300M-read kernel profile (bench line printed)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof300
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof300 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof300/bench.json 2> gpurun_out/prof300/bench.err || { tail -30 gpurun_out/prof300/bench.err; exit 1; }
cat gpurun_out/prof300/bench.json
