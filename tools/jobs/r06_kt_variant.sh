#!/bin/bash
# kernel trace of an engine build: tools/jobs/r06_kt_variant.sh LIB OUTNAME [bench args...]
cd "${GRAFT_REPO_ROOT:-$PWD}"
source tools/gpu_steps.sh
R=$PWD
lib=$1; out=$2; shift 2
mkdir -p gpurun_out/kt
step 300 "cd /tmp && export TMPDIR=/tmp && SAC_ENGINE_LIB=$R/soft-actor-critic_amd/$lib rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt/$out -o kt -- python3 $R/bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-sweep --no-bf16 --no-c3 $* > $R/gpurun_out/kt/$out.log 2>&1"
f=$(find gpurun_out/kt/$out -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/kt/${out}_stats.csv
find gpurun_out/kt/$out -name "*.db" -delete; find gpurun_out/kt/$out -name "*kernel_trace.csv" -delete
exit $STEP_RC
