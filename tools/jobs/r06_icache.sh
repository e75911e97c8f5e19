#!/bin/bash
# Round 6: instruction-cache counters of the phase kernels (SQC_ICACHE_* , SQ_IFETCH),
# C2 / C3 x fp32 / bf16 -> gpurun_out/r06/r06_icache_counters.txt
cd "${GRAFT_REPO_ROOT:-$PWD}"
source tools/gpu_steps.sh
mkdir -p gpurun_out/r06
IC="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES GRBM_GUI_ACTIVE"
names=""
for cp in "c2 fp32" "c2 bf16" "c3 fp32" "c3 bf16"; do
  set -- $cp
  step 200 "BENCH_ARGS='--precision $2 --config $1 --no-c3' bash tools/pmc_pass.sh ic_$1_$2 '$IC'"
  names="$names ic_$1_$2"
done
step 60 "python3 tools/pmc_read.py $names > gpurun_out/r06/r06_icache_counters.txt"
rm -rf gpurun_out/pmc
exit $STEP_RC
