# bf16 split layer-0 update tiles with summed dY parts (SAC_GSUM_BF16): parity, then C2 bf16 A/B
source tools/gpu_steps.sh
step 400 "python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py -v --timeout 200 --timeout-method thread -k 'bf16 or c2' > gpurun_out/r04_gsum_parity.log 2>&1"
run() { step 120 "$1 python bench.py --precision bf16 --steps 2000 --warmup 200 --no-cpu-baseline --no-sweep --no-bf16 --no-c3 2>/dev/null | python3 -c \"import json,sys; d=json.load(sys.stdin); print('$1', d['value'], [round(x*1e3,2) for x in d['phase_ms']])\" >> gpurun_out/r04_gsum_ab.txt"; }
rm -f gpurun_out/r04_gsum_ab.txt
for rep in 1 2; do
  run "SAC_GSUM_BF16=0"
  run "SAC_GSUM_BF16=1"
  run "SAC_GSUM_BF16=1 SAC_PI0_PARTS=1 SAC_Q0_PARTS=1"
done
exit $STEP_RC
