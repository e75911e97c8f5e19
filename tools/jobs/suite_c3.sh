# The GPU suite, then the C3 bench legs (both precisions) of the current build
source tools/gpu_steps.sh
step 900 "python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_suite.log 2>&1"
step 300 "python bench.py --config c3 --steps 250 --warmup 30 --no-cpu-baseline --no-sweep > gpurun_out/r04_c3.json 2> gpurun_out/r04_c3.err"
exit $STEP_RC
