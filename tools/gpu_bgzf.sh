# GPU: deflate tests + device BGZF throughput + kernel profile (sqlite -> top kernels)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-bgzf}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bgzf.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python tools/bgzf_bench.py 20000000 3 > $OUT/bench.json 2>&1 || { cat $OUT/bench.json; exit 1; }
grep GBps $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python tools/bgzf_bench.py 20000000 1 > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-5 "$f" | head -12
