#!/bin/bash
# deflate candidate-round A/B (OGE_DEFL_CAND_R) at 20M reads: GB/s and ratio (tools/bgzf_bench.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-defl_r}
mkdir -p $OUT
export TMPDIR=/tmp
for R in ${RS:-1 2 4 1}; do
  OGE_DEFL_CAND_R=$R timeout -k 10 300 python -u tools/bgzf_bench.py 20000000 3 > $OUT/r$R.json 2> $OUT/r$R.err || { tail -20 $OUT/r$R.err; exit 1; }
  echo "R=$R $(cat $OUT/r$R.json)"
done
