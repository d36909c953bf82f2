#!/bin/bash
# SQ counters of the deflate kernels (counter collection serialises the kernels: the CSV timestamps are
# isolated durations) over the 4M-read codec bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-pmcdefl}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "k_defl|k_infl" -d $OUT/p1 -o run --output-format csv -- python3 tools/bgzf_bench.py 4000000 1 > $OUT/p1.log 2>&1 || { tail -20 $OUT/p1.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM --kernel-include-regex "k_defl|k_infl" -d $OUT/p2 -o run --output-format csv -- python3 tools/bgzf_bench.py 4000000 1 > $OUT/p2.log 2>&1 || { tail -20 $OUT/p2.log; exit 1; }
echo done
