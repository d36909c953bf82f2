#!/bin/bash
# inflate by input compressor (tools/infl_src_ab.py), plain and under a rocprofv3 kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-infl_src}
N=${2:-20000000}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/infl_src_ab.py $N > $OUT/ab.json 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
cat $OUT/ab.json
