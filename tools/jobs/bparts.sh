# C3 batch-part counts of the update tiles (SAC_BPARTS) and the stage path, one box
source tools/gpu_steps.sh
for p in 2 3 4; do
  step 200 "SAC_BPARTS=$p python bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_bp${p}_c3.json 2> gpurun_out/r04_bp${p}_c3.err"
done
step 200 "SAC_WIDE=1 python bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_bpw_c3.json 2> gpurun_out/r04_bpw_c3.err"
step 200 "SAC_WIDE=1 python bench.py --config c3 --precision bf16 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_bpw_c3bf.json 2> gpurun_out/r04_bpw_c3bf.err"
step 200 "python bench.py --config c3 --precision bf16 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_bp3_c3bf.json 2> gpurun_out/r04_bp3_c3bf.err"
exit $STEP_RC
