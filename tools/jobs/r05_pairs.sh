# Pair-tile kernels (layout "pairs"): parity, then C3 steps/s against the
# default row-tile kernels on one box, both precisions, interleaved twice.
source tools/gpu_steps.sh
R=${GRAFT_REPO_ROOT:-$PWD}
S=$R/gpurun_out/${R05_OUT:-r05_pairs}
mkdir -p $S
step 600 "python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k 'pair' > $S/tests.log 2>&1"
for rep in 1 2; do
  for prec in fp32 bf16; do
    for lay in "" "layout=pairs"; do
      step 200 "python bench.py --config c3 --precision $prec --steps 300 --warmup 30 --no-cpu-baseline --no-sweep --no-bf16 --no-c3 ${lay:+--layout $lay} 2>/dev/null | python3 -c \"import json,sys; d=json.load(sys.stdin); print('$rep $prec ${lay:-rows}', d['value'], [round(x*1e3,2) for x in d['phase_ms']])\" >> $S/ab.txt"
    done
  done
done
exit $STEP_RC
