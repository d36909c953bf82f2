#!/bin/bash
# round 2: lane inflate + pipeline tests, small and full bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02
T="--maxfail=8 -v --timeout 120 --timeout-method thread"
timeout -k 10 400 python -u -m pytest tests/test_gpu_inflate.py $T > gpurun_out/r02/pytest_inflate.log 2>&1; rc=$?
tail -15 gpurun_out/r02/pytest_inflate.log
[ $rc -eq 0 ] || { echo "inflate tests failed rc=$rc"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_cli.py $T > gpurun_out/r02/pytest_pipeline.log 2>&1; rc=$?
tail -5 gpurun_out/r02/pytest_pipeline.log
[ $rc -eq 0 ] || { echo "pipeline tests failed rc=$rc"; grep -E "FAILED|Error" gpurun_out/r02/pytest_pipeline.log | head -20; exit 1; }
timeout -k 10 300 python -u bench.py --pairs 10000000 --steps 2 --no-realign --no-cpu-baseline > gpurun_out/r02/bench_20m.json 2> gpurun_out/r02/bench_20m.err || { echo "bench20 failed"; tail -20 gpurun_out/r02/bench_20m.err; exit 1; }
tail -4 gpurun_out/r02/bench_20m.err
timeout -k 10 800 python -u bench.py --steps 2 --kernel-steps 2 > gpurun_out/r02/bench_300m.json 2> gpurun_out/r02/bench_300m.err || { echo "bench300 failed"; tail -20 gpurun_out/r02/bench_300m.err; exit 1; }
tail -8 gpurun_out/r02/bench_300m.err
