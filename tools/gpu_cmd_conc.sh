set -o pipefail
OUT=gpurun_out/${1:-conc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/concurrency_lab.py 262144 single j2 f2 f4 j4 single > $OUT/conc_262144.jsonl 2> $OUT/err.log &&
timeout -k 10 300 python tools/concurrency_lab.py 65536 single j2 f2 f4 single > $OUT/conc_65536.jsonl 2>> $OUT/err.log &&
cat $OUT/*.jsonl
