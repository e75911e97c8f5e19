# usage: bash tools/jobs/flow.sh TAG -- flow-kernel tests and C3 benches
source tools/gpu_steps.sh
T=${1:-flow}
step 200 "python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread -k 'staged_batches_equal_fresh' > gpurun_out/r04_${T}_engine.log 2>&1"
step 400 "python -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k 'flow or stage_path or c3' > gpurun_out/r04_${T}_parity.log 2>&1"
step 200 "SAC_WIDE=1 SAC_WIDE_FLOW=1 python bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_${T}_c3.json 2> gpurun_out/r04_${T}_c3.err"
step 200 "SAC_WIDE=1 SAC_WIDE_FLOW=1 python bench.py --config c3 --precision bf16 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_${T}_c3bf.json 2> gpurun_out/r04_${T}_c3bf.err"
exit $STEP_RC
