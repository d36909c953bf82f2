#!/bin/bash
# r04g: codec tests + inflate timing (tools/gpu_r04f.sh), then deflate variants
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
VARS="openge_amd/_var/lib_r03.so" bash tools/gpu_r04f.sh $1 && VARS="openge_amd/_var/lib_tp1024.so" bash tools/gpu_defl_var.sh $1
