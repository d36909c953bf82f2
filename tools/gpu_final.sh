#!/bin/bash
# final round pass: GPU tests, smoke, default bench, rocprof kernel stats, PMC passes, then the CLI at 150M
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r02s3f}
bash tools/gpu_round3.sh $TAG && E2E_POOL=default bash tools/gpu_pool_ab.sh ${TAG}_cli
