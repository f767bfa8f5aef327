set -o pipefail
OUT=gpurun_out/${1:-render_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o r -f csv -- python3 tools/render_prof.py 64 20 > /dev/null 2> $OUT/err.log &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace1 -o r -f csv -- python3 tools/render_prof.py 1 20 > /dev/null 2>> $OUT/err.log &&
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-include-regex render_kernel -d $OUT/g0 -o p -f csv -- python3 tools/render_prof.py 64 5 > /dev/null 2>> $OUT/err.log &&
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU --kernel-include-regex render_kernel -d $OUT/g1 -o p -f csv -- python3 tools/render_prof.py 64 5 > /dev/null 2>> $OUT/err.log &&
grep render_kernel $OUT/trace/r_kernel_stats.csv $OUT/trace1/r_kernel_stats.csv | cut -c1-220 &&
python3 - $OUT <<'PY'
import csv, glob, sys, collections
for f in sorted(glob.glob(sys.argv[1] + "/g*/p_counter_collection.csv")):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print({k: round(sum(v) / len(v)) for k, v in acc.items()})
PY
