#!/bin/bash
# rocprofv3 kernel trace of the 300M-read kernel-only step (stages JSON on stdout)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-kprof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --kernel-only --kernel-steps 2 > $OUT/kstep.json 2> $OUT/kstep.err || { tail -20 $OUT/kstep.err; exit 1; }
cat $OUT/kstep.json
