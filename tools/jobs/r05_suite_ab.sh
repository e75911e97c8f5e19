# Full GPU suite (no -x: every failure listed), smoke, then a same-box A/B (R05_AB libs).
source tools/gpu_steps.sh
R=${GRAFT_REPO_ROOT:-$PWD}
S=$R/gpurun_out/${R05_OUT:-r05_suite}
mkdir -p $S
step 900 "python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $S/gputest.log 2>&1"
step 200 "python -c 'import __graft_entry__ as g; g.smoke()' > $S/smoke.log 2>&1"
[ -n "${R05_AB:-}" ] && step 500 "bash tools/ab_bench.sh ${R05_AB} > $S/ab.txt 2>&1"
exit $STEP_RC
