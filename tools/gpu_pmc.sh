# PMC passes (one rocprofv3 run per counter group) over the sort+dedup bench at 50M reads
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-pmc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-include-regex "k_input_pass|k_gather16|k_radix_scatter|k_meta_gather|k_ties|k_pair_runs" -d $OUT/$name -o run --output-format csv -- python3 bench.py --pairs 25000000 --steps 1 --warmup 0 --no-cpu-baseline --no-realign > $OUT/$name.json 2> $OUT/$name.err || { echo "pass $name failed"; tail -5 $OUT/$name.err; return 1; }
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE && \
run sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM && \
run tcc1 FETCH_SIZE && run tcc2 WRITE_SIZE
echo done
