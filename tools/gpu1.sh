set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu1.log 2>&1
rc=$?
tail -30 gpurun_out/gpu1.log
exit $rc
