set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-cli01}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cli.py -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_cli.log 2>&1 || { tail -40 $OUT/pytest_cli.log; exit 1; }
tail -3 $OUT/pytest_cli.log
timeout -k 10 600 python tools/e2e_cli.py 20000000 /tmp/e2e 16 > $OUT/e2e_20m.json 2>&1 || { cat $OUT/e2e_20m.json; exit 1; }
cat $OUT/e2e_20m.json
