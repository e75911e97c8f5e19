#!/bin/bash
# C3 (B = 4096) kernel trace, fp32 and bf16: per-kernel durations into gpurun_out/c3/
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
S=$R/gpurun_out/c3
rm -rf "$S" && mkdir -p "$S"
cd /tmp && export TMPDIR=/tmp
for p in fp32 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$S/kt_$p" -o kt -- python3 "$R/bench.py" --config c3 --precision $p \
    --steps ${STEPS:-300} --warmup 50 --no-cpu-baseline --no-sweep --no-bf16 > "$S/bench_$p.log" 2>&1
  f=$(find "$S/kt_$p" -name "*kernel_stats.csv" -print -quit); cp "$f" "$S/kernel_stats_c3_$p.csv"
  find "$S/kt_$p" -name "*.db" -delete
done
ls -la "$S"
