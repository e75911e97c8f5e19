# 64 x 64 update tiles at C3: batch-part counts (SAC_BPARTS) against SAC_TILE64=0, one box
source tools/gpu_steps.sh
T=${1:-t64b}
step 300 "SAC_TILE64=1 python -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k c3 > gpurun_out/r04_${T}_parity.log 2>&1"
for p in d 2 3 4 6; do
  E="SAC_TILE64=1"; [ "$p" != d ] && E="SAC_TILE64=1 SAC_BPARTS=$p"
  step 200 "$E python bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_${T}_p${p}.json 2> gpurun_out/r04_${T}_p${p}.err"
done
step 200 "python bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_${T}_32.json 2> gpurun_out/r04_${T}_32.err"
step 200 "SAC_TILE64=1 python bench.py --config c3 --precision bf16 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_${T}_bf.json 2> gpurun_out/r04_${T}_bf.err"
step 200 "python bench.py --config c3 --precision bf16 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_${T}_bf32.json 2> gpurun_out/r04_${T}_bf32.err"
exit $STEP_RC
