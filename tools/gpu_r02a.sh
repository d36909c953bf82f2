#!/bin/bash
# round-2 first GPU pass: pipeline + CLI tests, a small and a full-size bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_cli.py --maxfail=5 -v --timeout 120 --timeout-method thread > gpurun_out/r02/pytest_pipeline.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r02/pytest_pipeline.log; exit 1; }
tail -3 gpurun_out/r02/pytest_pipeline.log
timeout -k 10 300 python -u bench.py --pairs 10000000 --steps 2 --no-realign --no-cpu-baseline > gpurun_out/r02/bench_20m.json 2> gpurun_out/r02/bench_20m.err || { echo "bench20 failed"; tail -20 gpurun_out/r02/bench_20m.err; exit 1; }
cat gpurun_out/r02/bench_20m.json | head -c 1500; echo
timeout -k 10 800 python -u bench.py --steps 2 --kernel-steps 2 > gpurun_out/r02/bench_300m.json 2> gpurun_out/r02/bench_300m.err || { echo "bench300 failed"; tail -20 gpurun_out/r02/bench_300m.err; exit 1; }
tail -5 gpurun_out/r02/bench_300m.err
