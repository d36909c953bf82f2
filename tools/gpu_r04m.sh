#!/bin/bash
# r04m: codec tests (incl. the deflate pins) on the current library, deflate timing, Huffman phase clocks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04m}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bgzf.py tests/test_gpu_inflate.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest_codec.log 2>&1 || { tail -40 $OUT/pytest_codec.log; exit 1; }
tail -2 $OUT/pytest_codec.log
VARS= bash tools/gpu_defl_var.sh $1 || exit 1
for v in hx hx2; do
  timeout -k 10 200 python tools/diag_defl.py openge_amd/_var/lib_$v.so > $OUT/$v.txt 2>&1 || { tail -20 $OUT/$v.txt; exit 1; }
  grep "huff-exp\|deflate ms" $OUT/$v.txt | head -5
done
