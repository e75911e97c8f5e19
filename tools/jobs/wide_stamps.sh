source tools/gpu_steps.sh
step 300 'python -u tools/wide_stamps.py c3 fp32 > gpurun_out/r04_wide_stamps_fp32.txt 2>&1'
step 200 'python -u tools/wide_stamps.py c3 bf16 2 6 10 > gpurun_out/r04_wide_stamps_bf16.txt 2>&1'
step 200 'python bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_wide_c3b.json 2> gpurun_out/r04_wide_c3b.err'
exit $STEP_RC
