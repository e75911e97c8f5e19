#!/bin/bash
# Round-6 profile of the shipped build (each GPU step its own time limit):
#   kernel trace + FETCH_SIZE / WRITE_SIZE passes for C2 / C3 x fp32 / bf16
#   (gpurun_out/r06p_<cfg>_<prec>/), SQ passes (MFMA-busy, waits) -> gpurun_out/r06/r06_sq_counters.txt
cd "${GRAFT_REPO_ROOT:-$PWD}"
source tools/gpu_steps.sh
R=$PWD
mkdir -p gpurun_out/r06
for cp in "c2 fp32 1000" "c2 bf16 1000" "c3 fp32 250" "c3 bf16 250"; do
  set -- $cp
  step 420 "PROF_DIR=r06p_$1_$2 STEPS=$3 BENCH_ARGS='--config $1 --precision $2 --no-c3' bash tools/profile_round.sh > gpurun_out/r06/prof_$1_$2.log 2>&1"
  step 120 "python3 tools/pmc_summary.py r06 gpurun_out/r06p_$1_$2 --tag _$1_$2 --config $1 --precision $2 --dst gpurun_out/r06 > /dev/null && rm -rf gpurun_out/r06p_$1_$2"
done
SQA="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES"
SQB="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
for cp in "c2 fp32" "c2 bf16" "c3 fp32" "c3 bf16"; do
  set -- $cp
  step 200 "BENCH_ARGS='--precision $2 --config $1 --no-c3' bash tools/pmc_pass.sh sqa_$1_$2 '$SQA'"
  step 200 "BENCH_ARGS='--precision $2 --config $1 --no-c3' bash tools/pmc_pass.sh sqb_$1_$2 '$SQB'"
done
step 60 "python3 tools/pmc_read.py sqa_c2_fp32 sqb_c2_fp32 sqa_c2_bf16 sqb_c2_bf16 sqa_c3_fp32 sqb_c3_fp32 sqa_c3_bf16 sqb_c3_bf16 > gpurun_out/r06/r06_sq_counters.txt"
rm -rf gpurun_out/pmc
find gpurun_out -name "*.db" -size +20M -delete
exit $STEP_RC
