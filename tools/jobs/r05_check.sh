# Round-5 check of the current build on the GPU box: the GPU suite (tie-free
# parity draws print their redraw counts: -s), smoke, the default bench line,
# then rocprofv3 kernel stats + FETCH / WRITE / TCC hit-miss passes for the
# bf16 C2 and C3 steps (the missing bf16 evidence).
source tools/gpu_steps.sh
S=gpurun_out/${R05_OUT:-r05_check}
mkdir -p $S
step 900 "python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $S/gputest.log 2>&1"
step 200 "python -c 'import __graft_entry__ as g; g.smoke()' > $S/smoke.log 2>&1"
step 400 "python bench.py > $S/bench.json 2> $S/bench.err"
if [ -n "${R05_PROF:-}" ]; then
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for cfg in c2 c3; do
  A="--config $cfg --precision bf16 --no-cpu-baseline --no-sweep --no-bf16 --no-c3"
  step 200 "rocprofv3 --kernel-trace --stats -d $R/$S/kt_${cfg}_bf16 -o kt -- python3 $R/bench.py --steps 400 --warmup 50 $A > $R/$S/kt_${cfg}_bf16.log 2>&1"
  step 120 "rocprofv3 --pmc FETCH_SIZE -d $R/$S/fetch_${cfg}_bf16 -o p -- python3 $R/bench.py --steps 40 --warmup 8 $A > $R/$S/fetch_${cfg}_bf16.log 2>&1"
  step 120 "rocprofv3 --pmc WRITE_SIZE -d $R/$S/write_${cfg}_bf16 -o p -- python3 $R/bench.py --steps 40 --warmup 8 $A > $R/$S/write_${cfg}_bf16.log 2>&1"
  step 120 "rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $R/$S/tcc_${cfg}_bf16 -o p -- python3 $R/bench.py --steps 40 --warmup 8 $A > $R/$S/tcc_${cfg}_bf16.log 2>&1"
done
fi
exit $STEP_RC
