# 64 x 64 update tiles at C3: parity, engine tests, benches against SAC_TILE64=0
source tools/gpu_steps.sh
T=${1:-t64}
step 300 "python -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k 'c3 or rowtile or wide_deep or stage_b2000' > gpurun_out/r04_${T}_parity.log 2>&1"
step 300 "python -u -m pytest tests/test_gpu_engine.py -v --timeout 120 --timeout-method thread -k 'c3 or large_batch or stage_path' > gpurun_out/r04_${T}_engine.log 2>&1"
step 200 "python bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_${T}_c3.json 2> gpurun_out/r04_${T}_c3.err"
step 200 "python bench.py --config c3 --precision bf16 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_${T}_c3bf.json 2> gpurun_out/r04_${T}_c3bf.err"
step 200 "SAC_TILE64=0 python bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_${T}0_c3.json 2> gpurun_out/r04_${T}0_c3.err"
step 200 "SAC_WIDE=1 python bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_${T}w_c3.json 2> gpurun_out/r04_${T}w_c3.err"
exit $STEP_RC
