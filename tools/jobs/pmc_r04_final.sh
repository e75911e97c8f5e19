# Round-4 SQ counter passes (MFMA-busy + GRBM; wave / wait cycles) of the final build,
# C2 and C3, fp32 and bf16, each pass its own rocprofv3 run -> gpurun_out/r04/r04_sq_counters.txt
source tools/gpu_steps.sh
R=${GRAFT_REPO_ROOT:-$PWD}
S=$R/gpurun_out/r04
mkdir -p "$S"
SQA="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES"
SQB="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
for cp in "c2 fp32" "c2 bf16" "c3 fp32" "c3 bf16"; do
  set -- $cp
  step 200 "BENCH_ARGS='--precision $2 --config $1 --no-c3' bash tools/pmc_pass.sh sqa_$1_$2 '$SQA'"
  step 200 "BENCH_ARGS='--precision $2 --config $1 --no-c3' bash tools/pmc_pass.sh sqb_$1_$2 '$SQB'"
done
step 60 "python3 tools/pmc_read.py sqa_c2_fp32 sqb_c2_fp32 sqa_c2_bf16 sqb_c2_bf16 sqa_c3_fp32 sqb_c3_fp32 sqa_c3_bf16 sqb_c3_bf16 > $S/r04_sq_counters.txt"
rm -rf gpurun_out/pmc
exit $STEP_RC
