# Round-5: the GPU suite + smoke on the current build, a same-box A/B against the
# committed build (lib_base.so), and stamps of C2 per precision.
source tools/gpu_steps.sh
R=${GRAFT_REPO_ROOT:-$PWD}
S=$R/gpurun_out/${R05_OUT:-r05_val}
mkdir -p $S
step 900 "python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $S/gputest.log 2>&1"
step 200 "python -c 'import __graft_entry__ as g; g.smoke()' > $S/smoke.log 2>&1"
[ -n "${R05_BENCH:-}" ] && step 400 "python bench.py > $S/bench.json 2> $S/bench.err"
[ -n "${R05_AB:-}" ] && step 400 "bash tools/ab_bench.sh ${R05_AB} > $S/ab.txt 2>&1"
if [ -n "${R05_STAMPS:-}" ]; then
  for cp in ${R05_STAMPS}; do
    step 200 "python3 tools/stamps.py ${cp%%:*} ${cp##*:} > $S/stamps_${cp%%:*}_${cp##*:}.txt 2>&1"
  done
fi
exit $STEP_RC
