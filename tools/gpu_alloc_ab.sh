#!/bin/bash
# inflate with library-allocated buffers: OGE_ALLOC_CONTIG values (CONTIG, default "0 1": hipMalloc vs
# contiguous) x experiment builds (args: openge_amd/_var/lib_NAME.so; none = the default library), processes alternated
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-alloc_ab}; shift
mkdir -p $OUT
for rep in $(seq ${REPS:-2}); do
  for c in ${CONTIG:-0 1}; do
    for v in ${@:-default}; do
      lib=""; [ "$v" != default ] && lib=openge_amd/_var/lib_$v.so
      OGE_ALLOC_CONTIG=$c timeout -k 10 150 python -u tools/diag_infl_alloc.py $lib >> $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
    done
  done
done
grep contig= $OUT/ab.txt | cut -c1-200
