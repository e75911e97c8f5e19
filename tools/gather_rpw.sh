#!/bin/bash
# Gather sweep at several rows-per-wave settings (SAC_GATHER_RPW), interleaved twice
set -euo pipefail
for rep in 1 2; do
  for rpw in 16 8 4 32; do
    SAC_GATHER_RPW=$rpw timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-bf16 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('rpw $rpw', d['replay_gather_GBps_sweep'], d['replay_sample_GBps_sweep'])"
  done
done
