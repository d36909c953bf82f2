#!/bin/bash
# benches only: a small one, then the full 300M bench (args passed through to the second)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02
timeout -k 10 300 python -u bench.py --pairs 10000000 --steps 2 --no-realign --no-cpu-baseline > gpurun_out/r02/bench_20m.json 2> gpurun_out/r02/bench_20m.err || { echo "bench20 failed"; tail -20 gpurun_out/r02/bench_20m.err; exit 1; }
tail -4 gpurun_out/r02/bench_20m.err
timeout -k 10 900 python -u bench.py "$@" > gpurun_out/r02/bench_300m.json 2> gpurun_out/r02/bench_300m.err || { echo "bench300 failed"; tail -20 gpurun_out/r02/bench_300m.err; exit 1; }
tail -12 gpurun_out/r02/bench_300m.err
