#!/bin/bash
# One rocprofv3 --pmc pass over a short bench run: tools/pmc_pass.sh NAME "CTR1 CTR2 ..."
# Output: gpurun_out/pmc/NAME (rocpd database); summarise with tools/pmc_read.py NAME.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/pmc/$1
rm -rf "$OUT" && mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc $2 -d "$OUT" -o p -- python3 "$R/bench.py" --steps 40 --warmup 8 --no-cpu-baseline --no-sweep --no-bf16 ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
