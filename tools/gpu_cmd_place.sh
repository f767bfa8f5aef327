set -o pipefail
OUT=gpurun_out/${1:-place}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/placement_lab.py 262144 torch s0 s256 s4096 s65536 s69632 torch > $OUT/place_262144.jsonl 2> $OUT/err.log &&
timeout -k 10 400 python tools/placement_lab.py 16777216 torch s0 s256 s4096 s65536 s69632 torch > $OUT/place_16m.jsonl 2>> $OUT/err.log &&
cat $OUT/*.jsonl
