#!/bin/bash
# Round-6 closing run on the shipped build: the GPU suite, smoke, the bench in the
# driver's form (--steps 20 --warmup 5) and the builder's default form.
#   tools/jobs/r06_final.sh OUTDIR
cd "${GRAFT_REPO_ROOT:-$PWD}"
source tools/gpu_steps.sh
S=gpurun_out/${1:-r06_final}
mkdir -p $S
step 900 "python -u -m pytest tests -m gpu -q -rf -s --timeout 300 --timeout-method thread > $S/gputest.log 2>&1"
step 200 "python -c 'import __graft_entry__ as g; g.smoke()' > $S/smoke.log 2>&1"
step 300 "python bench.py --steps 20 --warmup 5 > $S/bench_driver_form.json 2> $S/bench_driver_form.err"
step 600 "python bench.py > $S/bench_default.json 2> $S/bench_default.err"
exit $STEP_RC
