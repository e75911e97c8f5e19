# C3 through the per-network role kernels past co-residency (SAC_ROLES=2) vs the one-block-per-row-tile kernels: parity, then A/B
source tools/gpu_steps.sh
step 300 "python -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k 'forced_role' > gpurun_out/r04_roles_parity.log 2>&1"
run() { step 200 "$1 python bench.py --config c3 --precision $2 --steps 200 --warmup 30 --no-cpu-baseline --no-sweep --no-bf16 2>/dev/null | python3 -c \"import json,sys; d=json.load(sys.stdin); print('$1 $2', d['value'], [round(x*1e3,2) for x in d['phase_ms']])\" >> gpurun_out/r04_roles_ab.txt"; }
rm -f gpurun_out/r04_roles_ab.txt
for rep in 1 2; do
  for p in fp32 bf16; do
    run "SAC_ROLES=1" $p
    run "SAC_ROLES=2" $p
  done
done
exit $STEP_RC
