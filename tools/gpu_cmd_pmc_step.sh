set -o pipefail
T=$1
mkdir -p gpurun_out/$T
WHAT=step ENVS=262144 REGEX=step_kernel timeout -k 10 600 bash tools/pmc_kernel.sh $T/pmc_step > gpurun_out/$T/pmc_step.txt 2>&1; rc=$?; tail -24 gpurun_out/$T/pmc_step.txt; exit $rc
