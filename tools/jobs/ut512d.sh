# C3 phase D as 512-thread update tiles (SAC_UPD_UT_D=512, two per CU, up to 8 batch parts) vs the 1024-thread default: parity, then A/B
source tools/gpu_steps.sh
step 400 "python -u -m pytest tests/test_gpu_parity.py -v --timeout 200 --timeout-method thread -k 'half_size or update_block_sizes or test_baseline_config_matches_oracle' > gpurun_out/r04_ut512d_parity.log 2>&1"
run() { step 200 "$1 python bench.py --config c3 --precision $2 --steps 200 --warmup 30 --no-cpu-baseline --no-sweep --no-bf16 2>/dev/null | python3 -c \"import json,sys; d=json.load(sys.stdin); print('$1 $2', d['value'], [round(x*1e3,2) for x in d['phase_ms']])\" >> gpurun_out/r04_ut512d_ab.txt"; }
rm -f gpurun_out/r04_ut512d_ab.txt
for rep in 1 2; do
  for p in fp32 bf16; do
    run "SAC_UPD_UT_D=1024" $p
    run "SAC_UPD_UT_D=512" $p
    run "SAC_UPD_UT_D=512 SAC_BPARTS_D=4" $p
    run "SAC_UPD_UT_D=512 SAC_BPARTS_D=8" $p
  done
done
exit $STEP_RC
