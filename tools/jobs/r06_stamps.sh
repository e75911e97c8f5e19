#!/bin/bash
# stamps of the C2 engine: tools/jobs/r06_stamps.sh OUTNAME [prec]
cd "${GRAFT_REPO_ROOT:-$PWD}"
source tools/gpu_steps.sh
step 300 "python3 tools/stamps.py c2 ${2:-fp32} > gpurun_out/$1_stamps_c2_${2:-fp32}.txt 2>&1"
exit $STEP_RC
