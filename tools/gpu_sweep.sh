# launch-shape sweep: sort/dedup parity tests, then bench stages for a few grid caps
# (env knobs read by records.hip)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-sweep}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for cfg in ${SWEEP:-"65536 2048" "131072 2048" "262144 2048"}; do
  set -- $cfg
  OGE_GATHER_BLOCKS=$1 OGE_INPUT_BLOCKS=$2 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-realign > $OUT/g$1_$2.json 2> $OUT/g$1_$2.err || { tail -5 $OUT/g$1_$2.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/g$1_$2.json')); print('gather', $1, 'input', $2, d['ms_per_step'], d['stages_ms']['gather_records'], d['stages_ms']['input_pass'])"
done
