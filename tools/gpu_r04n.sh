#!/bin/bash
# r04n: codec tests (incl. deflate pins), the restated-Huffman check, deflate timing, standalone kernel
# times (one stream) and the Huffman kernel's phase clocks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04n}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bgzf.py tests/test_gpu_inflate.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest_codec.log 2>&1 || { tail -40 $OUT/pytest_codec.log; exit 1; }
tail -2 $OUT/pytest_codec.log
VARS= bash tools/gpu_defl_var.sh $1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/dprof -o run --output-format csv -- python3 tools/diag_defl.py openge_amd/_var/lib_s1.so > $OUT/defl_s1.txt 2>&1 || { tail -20 $OUT/defl_s1.txt; exit 1; }
grep "deflate ms" $OUT/defl_s1.txt
timeout -k 10 200 python tools/diag_defl.py openge_amd/_var/lib_hx2.so > $OUT/hx2.txt 2>&1 || { tail -20 $OUT/hx2.txt; exit 1; }
grep "huff-exp" $OUT/hx2.txt | head -4
timeout -k 10 200 python tools/diag_defl.py openge_amd/_var/lib_px.so > $OUT/px.txt 2>&1 || { tail -20 $OUT/px.txt; exit 1; }
grep "parse-exp" $OUT/px.txt | head -4
