#!/bin/bash
# 300M bench at HEAD, then the same under rocprofv3 kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --steps 2 --kernel-steps 2 --no-cpu-baseline --no-realign > $OUT/bench_300m.json 2> $OUT/bench_300m.err || { echo "bench300 failed"; tail -20 $OUT/bench_300m.err; exit 1; }
tail -6 $OUT/bench_300m.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 -u bench.py --steps 2 --kernel-steps 1 --no-cpu-baseline --no-realign > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { echo "prof failed"; tail -20 $OUT/prof_bench.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
head -30 $OUT/kernel_stats.csv | cut -c1-160
