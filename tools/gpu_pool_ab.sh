#!/bin/bash
# CLI end to end at 150M reads with the device memory pool on / off / on (OGE_POOL), one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-pool_ab}
N=${2:-150000000}
mkdir -p $OUT
export TMPDIR=/tmp
df -h /tmp > $OUT/df.txt; free -g >> $OUT/df.txt
AVAIL=$(df --output=avail -B1G /tmp | tail -1 | tr -d ' ')
if [ "$AVAIL" -lt 65 ]; then echo "only ${AVAIL} GB free in /tmp"; exit 3; fi
E2E_POOL=${E2E_POOL:-1,0,1} timeout -k 10 900 python -u tools/e2e_cli.py $N /tmp/e2e 16 > $OUT/e2e.json 2> $OUT/e2e.err || { cat $OUT/e2e.err; cat $OUT/e2e.json; rm -rf /tmp/e2e; exit 1; }
cat $OUT/e2e.err; cat $OUT/e2e.json
rm -rf /tmp/e2e
