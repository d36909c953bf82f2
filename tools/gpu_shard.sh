set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-sh01}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py -x -v -m gpu --timeout 400 --timeout-method thread > $OUT/pytest_shard.log 2>&1 || { tail -40 $OUT/pytest_shard.log; exit 1; }
tail -3 $OUT/pytest_shard.log
OGE_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --pairs 2000000 > $OUT/bench2_gloo.json 2> $OUT/bench2_gloo.err || { tail -30 $OUT/bench2_gloo.err; exit 1; }
cat $OUT/bench2_gloo.json
timeout -k 10 900 python bench.py --no-cpu-baseline --no-realign > $OUT/bench1.json 2> $OUT/bench1.err || { tail -30 $OUT/bench1.err; exit 1; }
cat $OUT/bench1.json
