# Phase kernels skip the dead bias-partial stores (SAC_DBP_SKIP, default with the staged bias sums): GPU suite, then C2/C3 A/B
source tools/gpu_steps.sh
step 900 "python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_dbp_suite.log 2>&1"
run() { step 200 "$1 python bench.py --config $3 --precision $2 --steps $4 --warmup 30 --no-cpu-baseline --no-sweep --no-bf16 2>/dev/null | python3 -c \"import json,sys; d=json.load(sys.stdin); print('$1 $2 $3', d['value'], [round(x*1e3,2) for x in d['phase_ms']])\" >> gpurun_out/r04_dbp_ab.txt"; }
rm -f gpurun_out/r04_dbp_ab.txt
for rep in 1 2; do
  for p in fp32 bf16; do
    run "SAC_DBP_SKIP=0" $p c2 2000
    run "SAC_DBP_SKIP=1" $p c2 2000
    run "SAC_DBP_SKIP=0" $p c3 200
    run "SAC_DBP_SKIP=1" $p c3 200
  done
done
exit $STEP_RC
