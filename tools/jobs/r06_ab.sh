#!/bin/bash
# round 6: GPU suite (optional) + same-box A/B of engine builds
#   tools/jobs/r06_ab.sh OUTNAME [suite] -- lib1.so lib2.so ...
cd "${GRAFT_REPO_ROOT:-$PWD}"
source tools/gpu_steps.sh
out=$1; shift
mkdir -p gpurun_out
if [ "$1" = "suite" ]; then
  shift
  step 900 "python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/${out}_suite.txt 2>&1"
fi
[ "$1" = "--" ] && shift
[ $# -gt 0 ] && step 900 "tools/ab_bench.sh $* > gpurun_out/${out}_ab.txt 2>&1"
exit $STEP_RC
