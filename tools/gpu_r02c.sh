#!/bin/bash
# round 2 re-entry: whole GPU suite at HEAD, then the 300M bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02c
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 300 --timeout-method thread > gpurun_out/r02c/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r02c/pytest_gpu.log
[ $rc -eq 0 ] || { echo "gpu tests failed rc=$rc"; grep -E "FAILED|Error" gpurun_out/r02c/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 800 python -u bench.py --steps 2 --kernel-steps 2 --no-cpu-baseline > gpurun_out/r02c/bench_300m.json 2> gpurun_out/r02c/bench_300m.err || { echo "bench300 failed"; tail -20 gpurun_out/r02c/bench_300m.err; exit 1; }
tail -8 gpurun_out/r02c/bench_300m.err
