#!/bin/bash
# Round profile on the GPU box (run from the repo root via gpurun):
#   1. rocprofv3 --kernel-trace --stats of a bench run (per-kernel durations)
#   2. two separate --pmc passes (FETCH_SIZE, WRITE_SIZE) for HBM-side bytes
# Outputs under gpurun_out/prof/; tools/pmc_summary.py condenses them into profiles/.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${PROF_DIR:-prof}
rm -rf "$OUT" && mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps ${STEPS:-1000} --warmup 100 --no-cpu-baseline --no-sweep --no-bf16 ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt -- python3 "$R/bench.py" $ARGS > "$OUT/kt_bench.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch -- python3 "$R/bench.py" --steps 40 --warmup 8 --no-cpu-baseline --no-sweep --no-bf16 ${BENCH_ARGS:-} > "$OUT/fetch_bench.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write -- python3 "$R/bench.py" --steps 40 --warmup 8 --no-cpu-baseline --no-sweep --no-bf16 ${BENCH_ARGS:-} > "$OUT/write_bench.log" 2>&1
find "$OUT" -name "*.csv" | sort
