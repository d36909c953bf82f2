#!/bin/bash
# deflate + inflate SQ counters and kernel stats on a 2M-read stream (tools/bgzf_bench.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PMC_TAG=${1:-r02e}
bash tools/gpu_defl_pmc.sh > gpurun_out/defl_pmc.txt 2>&1 && bash tools/gpu_infl_pmc.sh > gpurun_out/infl_pmc.txt 2>&1; rc=$?
cat gpurun_out/defl_pmc.txt gpurun_out/infl_pmc.txt | cut -c1-400
exit $rc
