#!/bin/bash
# r04l: codec tests + inflate time (current), deflate kernels standalone (one stream) under a kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04l}
mkdir -p $OUT
export TMPDIR=/tmp
VARS= bash tools/gpu_r04f.sh $1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/dprof -o run --output-format csv -- python3 tools/diag_defl.py openge_amd/_var/lib_s1.so > $OUT/defl_s1.txt 2>&1 || { tail -20 $OUT/defl_s1.txt; exit 1; }
grep "deflate ms" $OUT/defl_s1.txt
f=$(find $OUT/dprof -name "*kernel_stats.csv" | head -1); head -8 $f | cut -c1-150
