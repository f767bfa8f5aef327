#!/bin/bash
# Counters per allocation at 16.8M drones (tools/lab/placement_pmc.py: three
# identical envs stepped in a fixed dispatch order).  Each pass is its own
# process (and placement); compare the envs within a pass.  Output:
# gpurun_out/place/.   bash tools/lab/placement_pmc.sh [pass ...]
set -o pipefail
O=gpurun_out/place; mkdir -p $O; export TMPDIR=/tmp
declare -A P
P[tlb]="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum"
P[utcl2]="GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
P[rdlat]="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum"
P[stall]="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum"
P[dram]="TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum"
P[wrlat]="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_LEVEL_sum"
for tag in "${@:-tlb utcl2}"; do
  timeout -s KILL 180 rocprofv3 --pmc ${P[$tag]} --kernel-include-regex step_kernel -d $O/pmc_$tag -o pmc -f csv \
    -- python3 tools/lab/placement_pmc.py 10 > $O/placement_$tag.jsonl 2> $O/placement_$tag.err || exit 1
  echo "== $tag"; cat $O/placement_$tag.jsonl
done
