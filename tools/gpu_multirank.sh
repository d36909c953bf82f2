# multi-rank rehearsal on one GPU: realign GPU tests, then bench.py under torchrun with 2 ranks
# sharing the card (gloo collectives; the driver's N-GPU runs use RCCL)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-multirank}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_realign.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_rl.log 2>&1 || { tail -30 $OUT/pytest_rl.log; exit 1; }
tail -1 $OUT/pytest_rl.log
OGE_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --pairs 10000000 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench2.json 2> $OUT/bench2.err || { tail -30 $OUT/bench2.err; exit 1; }
cat $OUT/bench2.json
