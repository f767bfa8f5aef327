# Round 2, call c: sensitivity lab (trig / sqrt / obs division / launch floors), rollout lab, short bench runs.
set -o pipefail
T=${1:-r02c}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --hbm-point 0 --rollout-point 0 --no-extra-points > gpurun_out/$T/bench_k20_$r.json 2>> gpurun_out/$T/bench.err || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('k20', d['value'], d['ms_per_step'], d['gpu_ms_per_step'], d['roofline']['frac'])" gpurun_out/$T/bench_k20_$r.json
done
timeout -k 10 600 python -u tools/kernel_lab.py --variants base,faketrig,fakesqrt,obsmul,nomath,empty,b512,b1024,emptyb1024 --envs 262144,16777216 --rounds 9 > gpurun_out/$T/lab.jsonl 2> gpurun_out/$T/lab.err; rc=$?; cat gpurun_out/$T/lab.jsonl; tail -3 gpurun_out/$T/lab.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/rollout_lab.py --variants base,faketrig,fakesqrt,obsmul,nomath --envs 65536,262144 --rounds 7 > gpurun_out/$T/rlab.jsonl 2> gpurun_out/$T/rlab.err; rc=$?; cat gpurun_out/$T/rlab.jsonl; tail -3 gpurun_out/$T/rlab.err; exit $rc
