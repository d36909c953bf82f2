#!/bin/bash
# the round's profiles without the bench line: rocprofv3 kernel stats of a short bench, then FETCH_SIZE /
# WRITE_SIZE / SQ_INSTS_VALU passes over one e2e step (input build + step: k_defl runs twice, k_infl once);
# summarise with STAGES="k_defl=2,k_infl=1,k_infl_huff=1,k_infl_lz=1" python tools/pmc_summary.py gpurun_out/TAG profiles/TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pcie > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { tail -30 $OUT/prof_bench.err; exit 1; }
for C in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-include-regex "k_defl|k_infl|k_gather16|k_input_pass|k_mate" -d $OUT/pmc_$C -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --e2e-only --no-cpu-baseline --no-realign --no-pcie > $OUT/pmc_$C.json 2> $OUT/pmc_$C.err || { tail -20 $OUT/pmc_$C.err; exit 1; }
done
echo done
