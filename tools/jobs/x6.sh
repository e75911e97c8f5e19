# split-MFMA (bf16x6) stage path: parity with the fp32 tolerances unchanged, then C3 benches
source tools/gpu_steps.sh
T=${1:-x6}
L=$PWD/soft-actor-critic_amd/libsac_engine_x6.so
step 400 "SAC_ENGINE_LIB=$L SAC_WIDE=1 python -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k 'c3 or wide or obs300 or stage or flow' > gpurun_out/r04_${T}_parity.log 2>&1"
step 200 "SAC_ENGINE_LIB=$L SAC_WIDE=1 python bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_${T}_c3.json 2> gpurun_out/r04_${T}_c3.err"
step 200 "SAC_WIDE=1 python bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_${T}_c3w.json 2> gpurun_out/r04_${T}_c3w.err"
step 200 "python bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline --no-sweep --no-bf16 > gpurun_out/r04_${T}_c3r.json 2> gpurun_out/r04_${T}_c3r.err"
exit $STEP_RC
