set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof1
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python3 bench.py --pairs 25000000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof1/bench.json 2> gpurun_out/prof1/bench.err || { tail -30 gpurun_out/prof1/bench.err; exit 1; }
cat gpurun_out/prof1/bench.json
find gpurun_out/prof1 -name "*stats*" | head
f=$(find gpurun_out/prof1 -name "*kernel_stats.csv" | head -1); head -40 "$f"
