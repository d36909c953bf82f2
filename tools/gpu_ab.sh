# A/B of env knobs on the bench stages: bash tools/gpu_ab.sh TAG "ENV=.. ENV2=.." "ENV=.." ...
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1
shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-realign > $OUT/ab$i.json 2> $OUT/ab$i.err || { tail -5 $OUT/ab$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/ab$i.json')); print('$cfg', d['ms_per_step'], d['stages_ms']['input_pass'])"
done
