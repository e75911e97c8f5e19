# usage: bash tools/jobs/wide.sh TAG  -- stage-path tests, stamps and C3 benches
source tools/gpu_steps.sh
T=${1:-wide}
step 300 "python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread -k 'stage_path or c3 or large_batch' > gpurun_out/r04_${T}_engine.log 2>&1"
step 500 "python -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k 'c3 or rowtile or wide or obs300 or stage_path' > gpurun_out/r04_${T}_parity.log 2>&1"
step 300 "python -u tools/wide_stamps.py c3 fp32 > gpurun_out/r04_${T}_stamps_fp32.txt 2>&1"
step 200 "python bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_${T}_c3.json 2> gpurun_out/r04_${T}_c3.err"
step 200 "python bench.py --config c3 --precision bf16 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_${T}_c3bf.json 2> gpurun_out/r04_${T}_c3bf.err"
[ -n "$2" ] && step 200 "SAC_WIDE=0 python bench.py --config c3 --precision bf16 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_rt_c3bf.json 2> gpurun_out/r04_rt_c3bf.err"
exit $STEP_RC
