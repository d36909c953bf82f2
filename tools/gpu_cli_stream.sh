#!/bin/bash
# CLI tests (incl. the streamed reader), then the 150M-read CLI end to end (streamed, then the host-copy reader)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-cli_stream}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cli.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
E2E_POOL=default bash tools/gpu_pool_ab.sh ${1:-cli_stream}_e2e && OGE_READER=hostcopy E2E_POOL=default bash tools/gpu_pool_ab.sh ${1:-cli_stream}_e2e_host
