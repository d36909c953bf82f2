#!/bin/bash
# r03 measurement: smoke, default bench, rocprofv3 kernel stats of the bench, and per-counter PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ_INSTS_VALU) over one e2e step (input build + step: k_defl runs twice,
# k_infl once).  Usage: gpu_r03b.sh TAG [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r03b}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cut -c1-1500 $OUT/bench.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pcie --no-realign "$@" > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { tail -30 $OUT/prof_bench.err; exit 1; }
for C in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
  timeout -s KILL 400 rocprofv3 --pmc $C --kernel-include-regex "k_defl|k_infl|k_gather16|k_input_pass" -d $OUT/pmc_$C -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --e2e-only --no-cpu-baseline --no-realign --no-pcie "$@" > $OUT/pmc_$C.json 2> $OUT/pmc_$C.err || { tail -20 $OUT/pmc_$C.err; exit 1; }
done
echo done
