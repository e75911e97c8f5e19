#!/bin/bash
# Round-2 profile set on the GPU box (run from the repo root via gpurun):
#   fp32 (headline) and bf16 C2: kernel trace + FETCH_SIZE / WRITE_SIZE passes
#   SQ pass (MFMA busy, wave/wait cycles) for fp32 and bf16 C2 and fp32/bf16 C3
#   replay gather at B = 1,048,576: kernel trace + FETCH / WRITE passes
# Summaries go to gpurun_out/r02/ (then copied into profiles/); the raw rocpd
# databases are deleted on the box (they exceed gpurun's 64 MiB copy-back).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
S=$R/gpurun_out/r02
mkdir -p "$S/logs"
step() { echo "[$(date +%T)] $*"; }
step fp32 c2; PROF_DIR=prof_fp32 BENCH_ARGS="--precision fp32" bash tools/profile_round.sh
python3 tools/pmc_summary.py r02 gpurun_out/prof_fp32 --tag _c2_fp32 --config c2 --precision fp32 --dst "$S" > /dev/null
step bf16 c2; PROF_DIR=prof_bf16 BENCH_ARGS="--precision bf16" bash tools/profile_round.sh
python3 tools/pmc_summary.py r02 gpurun_out/prof_bf16 --tag _c2_bf16 --config c2 --precision bf16 --dst "$S" > /dev/null
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
for cp in "c2 fp32" "c2 bf16" "c3 fp32" "c3 bf16"; do
  set -- $cp
  step sq $1 $2; BENCH_ARGS="--precision $2 --config $1" bash tools/pmc_pass.sh sq_$1_$2 "$SQ"
done
python3 tools/pmc_read.py sq_c2_fp32 sq_c2_bf16 sq_c3_fp32 sq_c3_bf16 > "$S/r02_sq_counters.txt"
step gather; bash tools/profile_gather.sh
python3 tools/pmc_summary.py r02 gpurun_out/prof_gather --tag _gather --config gather --precision fp32 --dst "$S" > /dev/null
find gpurun_out -name "*.log" -path "*prof*" -exec sh -c 'cp "$1" "$2/logs/$(echo "$1" | tr / _)"' _ {} "$S" \;
find gpurun_out -name "*.log" -path "*pmc*" -exec sh -c 'cp "$1" "$2/logs/$(echo "$1" | tr / _)"' _ {} "$S" \;
rm -rf gpurun_out/prof_fp32 gpurun_out/prof_bf16 gpurun_out/prof_gather gpurun_out/pmc
step profile_r02 done; ls -la "$S"
