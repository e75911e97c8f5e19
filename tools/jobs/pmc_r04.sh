# Round-4 counter set (run from the repo root via gpurun): for C2 and C3, fp32 and
# bf16, two separate rocprofv3 --pmc passes of a short bench run (SQ MFMA-busy +
# GRBM; SQ wave / wait cycles), plus a kernel trace and FETCH / WRITE passes for
# the fp32 headline.  Summaries -> gpurun_out/r04/ (raw databases deleted).
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
for c in c2 c3; do
  step 400 "PROF_DIR=prof_$c STEPS=400 BENCH_ARGS='--precision fp32 --config $c --no-c3' bash tools/profile_round.sh"
  step 60 "python3 tools/pmc_summary.py r04 gpurun_out/prof_$c --tag _${c}_fp32 --config $c --precision fp32 --dst $S > /dev/null"
done
cp gpurun_out/pmc/*/bench.log "$S/" 2>/dev/null || true
for d in gpurun_out/pmc/*; do cp "$d/bench.log" "$S/$(basename $d)_bench.log" 2>/dev/null || true; done
rm -rf gpurun_out/pmc gpurun_out/prof_c2 gpurun_out/prof_c3
ls -la "$S"
exit $STEP_RC
