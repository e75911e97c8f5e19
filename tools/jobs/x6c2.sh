# bf16x6 split MFMA in the split kernels (C2): fp32 parity suites with the x6 build, then A/B
source tools/gpu_steps.sh
T=${1:-x6c2}
L=$PWD/soft-actor-critic_amd/libsac_engine_x6.so
step 600 "SAC_ENGINE_LIB=$L python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_rng.py tests/test_gpu_ref_pins.py -v --timeout 200 --timeout-method thread > gpurun_out/r04_${T}_parity.log 2>&1"
step 600 "AB_ARGS='--no-c3 --no-bf16' bash tools/ab_bench.sh libsac_engine.so libsac_engine_x6.so > gpurun_out/r04_${T}_ab.txt 2>&1"
exit $STEP_RC
