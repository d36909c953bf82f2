#!/bin/bash
# rocprofv3 kernel trace of the e2e bench leg (small size) -> gpurun_out/r02/prof_e2e
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02
PAIRS=${1:-10000000}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r02/prof_e2e -o prof --output-format csv -- python3 -u bench.py --pairs $PAIRS --e2e-only --steps 2 --warmup 1 > gpurun_out/r02/prof_e2e.json 2> gpurun_out/r02/prof_e2e.err || { echo "prof failed"; tail -20 gpurun_out/r02/prof_e2e.err; exit 1; }
f=$(find gpurun_out/r02/prof_e2e -name "*kernel_stats.csv" | head -1)
head -25 "$f" | cut -d, -f1-8
