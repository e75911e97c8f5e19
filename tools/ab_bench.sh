#!/bin/bash
# A/B timing of engine builds on ONE box: tools/ab_bench.sh lib1.so lib2.so ... (fp32 C2 bench legs,
# interleaved twice so clock drift between runs shows)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
for rep in 1 2; do
  for lib in "$@"; do
    v=$(SAC_ENGINE_LIB=$R/soft-actor-critic_amd/$lib timeout -k 10 200 python3 $R/bench.py --steps 2000 --warmup 200 --no-cpu-baseline --no-sweep ${AB_ARGS:-} 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d.get('value_bf16'), d.get('value_c3'), d.get('value_c3_bf16'), [round(x*1e3,2) for x in d['phase_ms']])")
    echo "$rep $lib $v"
  done
done
