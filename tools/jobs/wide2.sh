source tools/gpu_steps.sh
step 500 'python -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k "c3 or rowtile or wide or obs300 or stage_path" > gpurun_out/r04_wide2_parity.log 2>&1'
step 300 'python -u tools/wide_stamps.py c3 fp32 > gpurun_out/r04_wide_stamps_fp32.txt 2>&1'
step 200 'python bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_wide_c3b.json 2> gpurun_out/r04_wide_c3b.err'
step 200 'python bench.py --config c3 --precision bf16 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_wide_c3bfb.json 2> gpurun_out/r04_wide_c3bfb.err'
exit $STEP_RC
