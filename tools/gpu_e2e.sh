# End-to-end `openge mergesort -M` on a C2-shaped BAM, BAM -> BAM.  The box has 79 GB of disk and a
# 300M-read C2 BAM is ~58 GB in + ~60 GB out, so the default is 150M reads (input + output ~59 GB).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-e2e300}
N=${2:-150000000}
mkdir -p $OUT
export TMPDIR=/tmp
df -h /tmp > $OUT/df.txt; free -g >> $OUT/df.txt; cat $OUT/df.txt
AVAIL=$(df --output=avail -B1G /tmp | tail -1 | tr -d ' ')
if [ "$AVAIL" -lt 65 ]; then echo "only ${AVAIL} GB free in /tmp"; exit 3; fi
timeout -k 10 900 python -u tools/e2e_cli.py $N /tmp/e2e 16 > $OUT/e2e.json 2> $OUT/e2e.err || { cat $OUT/e2e.err; cat $OUT/e2e.json; exit 1; }
cat $OUT/e2e.err; cat $OUT/e2e.json
rm -rf /tmp/e2e
