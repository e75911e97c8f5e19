# Bias gradients from the staged dY rows (TileDesc.bstage, default at Bp > 1024) vs the row tiles' partials: parity, then C3 and C2 A/B
source tools/gpu_steps.sh
step 600 "python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py -v --timeout 200 --timeout-method thread -k 'c3 or c2 or bias_gradient or large or staged_batch' > gpurun_out/r04_bstage_parity.log 2>&1"
run() { step 200 "$1 python bench.py --config $3 --precision $2 --steps $4 --warmup 30 --no-cpu-baseline --no-sweep --no-bf16 2>/dev/null | python3 -c \"import json,sys; d=json.load(sys.stdin); print('$1 $2 $3', d['value'], [round(x*1e3,2) for x in d['phase_ms']])\" >> gpurun_out/r04_bstage_ab.txt"; }
rm -f gpurun_out/r04_bstage_ab.txt
for rep in 1 2; do
  for p in fp32 bf16; do
    run "SAC_BIAS_STAGED=0" $p c3 200
    run "SAC_BIAS_STAGED=1" $p c3 200
    run "SAC_BIAS_STAGED=0" $p c2 2000
    run "SAC_BIAS_STAGED=1" $p c2 2000
  done
done
exit $STEP_RC
