#!/bin/bash
# deflate literal-batch A/B (OGE_DEFL_LITB) at 20M reads: GB/s and ratio (tools/bgzf_bench.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-defl_litb}
mkdir -p $OUT
export TMPDIR=/tmp
for B in ${LITBS:-1 2 4 1}; do
  OGE_DEFL_LITB=$B timeout -k 10 300 python -u tools/bgzf_bench.py 20000000 3 > $OUT/b$B.json 2> $OUT/b$B.err || { tail -20 $OUT/b$B.err; exit 1; }
  echo "LITB=$B $(cat $OUT/b$B.json)"
done
