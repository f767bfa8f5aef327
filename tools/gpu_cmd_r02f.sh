# Round 2, call f: separate graphs on separate streams (queues_lab.py).
set -o pipefail
OUT=gpurun_out/r02f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/queues_lab.py 262144 50 single q2 q4 d2 > $OUT/q_262144_50.jsonl 2> $OUT/q.err && cat $OUT/q_262144_50.jsonl &&
timeout -k 10 300 python -u tools/queues_lab.py 262144 20 single q2 q4 > $OUT/q_262144_20.jsonl 2>> $OUT/q.err && cat $OUT/q_262144_20.jsonl &&
timeout -k 10 300 python -u tools/queues_lab.py 1048576 50 single q2 q4 > $OUT/q_1m_50.jsonl 2>> $OUT/q.err && cat $OUT/q_1m_50.jsonl
