#!/bin/bash
# round measurement: GPU tests, smoke, default bench; with PROF=1 also the rocprofv3 kernel stats of a short
# bench and FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU passes over one e2e step (input build + step: k_defl
# runs twice, k_infl once)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
fi
timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cut -c1-700 $OUT/bench.json
if [ -n "$PROF" ]; then
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pcie > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { tail -30 $OUT/prof_bench.err; exit 1; }
for C in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
  timeout -s KILL 400 rocprofv3 --pmc $C --kernel-include-regex "k_defl|k_infl|k_gather16|k_input_pass" -d $OUT/pmc_$C -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --e2e-only --no-cpu-baseline --no-realign --no-pcie > $OUT/pmc_$C.json 2> $OUT/pmc_$C.err || { tail -20 $OUT/pmc_$C.err; exit 1; }
done
fi
echo done
