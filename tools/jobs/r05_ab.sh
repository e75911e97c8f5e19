# Parity subset + same-box A/B of engine builds: R05_K (pytest -k), R05_AB (libs), R05_STAMPS (cfg:prec ...)
source tools/gpu_steps.sh
R=${GRAFT_REPO_ROOT:-$PWD}
S=$R/gpurun_out/${R05_OUT:-r05_ab}
mkdir -p $S
[ -n "${R05_K:-}" ] && step 600 "python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k '${R05_K}' > $S/tests.log 2>&1"
[ -n "${R05_AB:-}" ] && step 500 "bash tools/ab_bench.sh ${R05_AB} > $S/ab.txt 2>&1"
if [ -n "${R05_STAMPS:-}" ]; then
  for cp in ${R05_STAMPS}; do
    step 200 "python3 tools/stamps.py ${cp%%:*} ${cp##*:} > $S/stamps_${cp%%:*}_${cp##*:}.txt 2>&1"
  done
fi
exit $STEP_RC
