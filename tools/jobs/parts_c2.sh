# C2 fp32: batch parts of the hidden-split layer-0 update tiles (SAC_PI0_PARTS / SAC_Q0_PARTS), interleaved twice
source tools/gpu_steps.sh
run() { step 120 "$1 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline --no-sweep --no-bf16 --no-c3 2>/dev/null | python3 -c \"import json,sys; d=json.load(sys.stdin); print('$1', d['value'], [round(x*1e3,2) for x in d['phase_ms']])\" >> gpurun_out/r04_parts_c2.txt"; }
rm -f gpurun_out/r04_parts_c2.txt
for rep in 1 2; do
  run "SAC_PI0_PARTS=2"
  run "SAC_PI0_PARTS=3"
  run "SAC_PI0_PARTS=4"
  run "SAC_PI0_PARTS=4 SAC_Q0_PARTS=3"
  run "SAC_Q0_PARTS=3"
done
exit $STEP_RC
