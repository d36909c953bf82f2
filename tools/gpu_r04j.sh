#!/bin/bash
# r04j: per-kernel times of the 300M e2e step (kernel trace) and the inflate kernels' SQ counters at 20M
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04j}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --e2e-only --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { tail -30 $OUT/prof_bench.err; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); head -25 $f | cut -c1-200
PMC_TAG=$1 bash tools/gpu_infl_pmc2.sh > $OUT/inflpmc.json
