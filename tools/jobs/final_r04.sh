# Round-4 final checks on one box: the GPU test suite, smoke(), the default bench
# line, and the kernel trace + FETCH / WRITE passes of the C2 fp32 headline and of C3 fp32.
source tools/gpu_steps.sh
S=gpurun_out/r04_final
mkdir -p $S
step 900 "python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $S/gputest.log 2>&1"
step 200 "python -c 'import __graft_entry__ as g; g.smoke()' > $S/smoke.log 2>&1"
step 400 "python bench.py > $S/bench.json 2> $S/bench.err"
step 500 "PROF_DIR=prof_c2f STEPS=1000 BENCH_ARGS='--precision fp32 --config c2 --no-c3' bash tools/profile_round.sh"
step 60 "python3 tools/pmc_summary.py r04 gpurun_out/prof_c2f --tag _c2_fp32_final --config c2 --precision fp32 --dst $S > /dev/null"
rm -rf gpurun_out/prof_c2f
step 500 "PROF_DIR=prof_c3f STEPS=150 BENCH_ARGS='--precision fp32 --config c3 --no-c3' bash tools/profile_round.sh"
step 60 "python3 tools/pmc_summary.py r04 gpurun_out/prof_c3f --tag _c3_fp32_final --config c3 --precision fp32 --dst $S > /dev/null"
rm -rf gpurun_out/prof_c3f
exit $STEP_RC
