#!/bin/bash
# phase-2 variant A/B at 100M reads, alternating builds in separate processes on one box:
#   bash tools/gpu_lz_ab.sh TAG VARIANT... (openge_amd/_var/lib_VARIANT.so, tools/build_variant.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for rep in 1 2; do
  for v in "$@"; do
    DIAG_READS=${DIAG_READS:-100000000} timeout -k 10 150 python -u tools/diag_infl.py openge_amd/_var/lib_$v.so >> gpurun_out/$TAG/ab.txt 2>&1 || exit 1
  done
done
grep reads gpurun_out/$TAG/ab.txt
