#!/bin/bash
# A/B timing of environment settings on ONE box: tools/ab_env.sh "SAC_X=0" "SAC_X=1" ...
# (bench legs with AB_ARGS, interleaved twice so clock drift between runs shows)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
for rep in 1 2; do
  for e in "$@"; do
    v=$(env $e timeout -k 10 200 python3 $R/bench.py --steps ${AB_STEPS:-2000} --warmup 200 --no-cpu-baseline --no-sweep ${AB_ARGS:-} 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d.get('value_bf16'), [round(x*1e3,2) for x in d['phase_ms']])")
    echo "$rep $e $v"
  done
done
