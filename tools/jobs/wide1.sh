source tools/gpu_steps.sh
step 400 'python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "c3 or rowtile" > gpurun_out/r04_wide_parity.log 2>&1'
step 120 'python bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep > gpurun_out/r04_wide_c3.json 2> gpurun_out/r04_wide_c3.err'
step 120 'python bench.py --config c3 --precision bf16 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep > gpurun_out/r04_wide_c3bf.json 2> gpurun_out/r04_wide_c3bf.err'
exit $STEP_RC
