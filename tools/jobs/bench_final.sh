# smoke() and the default bench line of the shipped build
source tools/gpu_steps.sh
S=gpurun_out/r04_final2
mkdir -p $S
step 200 "python -c 'import __graft_entry__ as g; g.smoke()' > $S/smoke.log 2>&1"
step 400 "python bench.py > $S/bench.json 2> $S/bench.err"
exit $STEP_RC
