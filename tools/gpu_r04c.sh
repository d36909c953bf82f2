#!/bin/bash
# r04c: deflate pins (sha golden, restated Huffman builder), the phase-1 v2 inflate's codec tests, then
# inflate stage times at 20M reads: v2 (default) vs r03's decoder vs r03 without long-literal lookups
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04c}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bgzf.py -x -v --timeout 200 --timeout-method thread -k "pinned or restated" > $OUT/pytest_pins.log 2>&1 || { tail -40 $OUT/pytest_pins.log; exit 1; }
tail -2 $OUT/pytest_pins.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_bgzf.py -x -v --timeout 200 --timeout-method thread --deselect tests/test_gpu_bgzf.py::test_deflate_bytes_pinned > $OUT/pytest_codec.log 2>&1 || { tail -40 $OUT/pytest_codec.log; exit 1; }
tail -2 $OUT/pytest_codec.log
bash tools/gpu_infl_var.sh $1
