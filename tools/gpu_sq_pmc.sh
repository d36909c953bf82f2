#!/bin/bash
# SQ counters of the phase-1 / phase-2 inflate kernels at 20M reads (tools/diag_infl.py), for the default
# library and for each openge_amd/_var/lib_*.so given as arguments; one rocprofv3 pass per counter group.
# KRE / DIAG select other kernels and driver (KRE=k_defl DIAG=tools/diag_defl.py: the deflate kernels)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
KRE=${KRE:-k_infl}
DIAG=${DIAG:-tools/diag_infl.py}
OUT=gpurun_out/${PMC_TAG:-sq}/${KRE}pmc
mkdir -p $OUT
export TMPDIR=/tmp
G1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH"
G2="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT"
for lib in default "$@"; do
  n=$(basename $lib .so)
  arg=""; [ "$lib" != default ] && arg=$lib
  for g in 1 2; do
    eval C=\$G$g
    timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "$KRE" -d $OUT/$n/p$g -o run --output-format csv -- python3 $DIAG $arg > $OUT/$n.p$g.txt 2>&1 || { tail -20 $OUT/$n.p$g.txt; exit 1; }
  done
done
python3 - $OUT <<'PY'
import csv, glob, sys, json
d = sys.argv[1]
res = {}
for f in glob.glob(d + "/*/p*/**/*counter_collection.csv", recursive=True):
    lib = f[len(d) + 1:].split("/")[0]
    for r in csv.DictReader(open(f)):
        import re
        m = re.search(r"(k_[a-z]+_\w+)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:40]
        res.setdefault(lib, {}).setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
out = {lib: {k: {c: sum(v) / len(v) * 0 + sum(v) for c, v in kv.items()} for k, kv in ks.items()} for lib, ks in res.items()}
print(json.dumps(out, indent=1))
PY
