#!/bin/bash
# Gather roofline evidence on the GPU box (run from the repo root via gpurun):
# kernel trace + separate FETCH_SIZE / WRITE_SIZE passes of tools/gather_bench.py.
# Then: python tools/pmc_summary.py r02 gpurun_out/prof_gather --tag _gather --config gather --precision fp32
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/prof_gather
rm -rf "$OUT" && mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt -- python3 "$R/tools/gather_bench.py" 20 1048576 > "$OUT/kt_bench.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch -- python3 "$R/tools/gather_bench.py" 5 1048576 > "$OUT/fetch_bench.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write -- python3 "$R/tools/gather_bench.py" 5 1048576 > "$OUT/write_bench.log" 2>&1
find "$OUT" -name "*.db" | sort
