# Round-5 baseline on the GPU box: the parity tests with tie-free draws, the
# default bench line of the round-start build, then rocprofv3 kernel stats +
# FETCH / WRITE / TCC hit-miss passes for the bf16 C2 and C3 steps (VERDICT r04
# item 3: the missing bf16 evidence).
source tools/gpu_steps.sh
S=gpurun_out/r05_base
mkdir -p $S
step 600 "python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 300 --timeout-method thread > $S/parity.log 2>&1"
step 400 "python bench.py > $S/bench.json 2> $S/bench.err"
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for cfg in c2 c3; do
  A="--config $cfg --precision bf16 --no-cpu-baseline --no-sweep --no-bf16 --no-c3"
  step 200 "rocprofv3 --kernel-trace --stats -d $R/$S/kt_${cfg}_bf16 -o kt -- python3 $R/bench.py --steps 400 --warmup 50 $A > $R/$S/kt_${cfg}_bf16.log 2>&1"
  step 120 "rocprofv3 --pmc FETCH_SIZE -d $R/$S/fetch_${cfg}_bf16 -o p -- python3 $R/bench.py --steps 40 --warmup 8 $A > $R/$S/fetch_${cfg}_bf16.log 2>&1"
  step 120 "rocprofv3 --pmc WRITE_SIZE -d $R/$S/write_${cfg}_bf16 -o p -- python3 $R/bench.py --steps 40 --warmup 8 $A > $R/$S/write_${cfg}_bf16.log 2>&1"
  step 120 "rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $R/$S/tcc_${cfg}_bf16 -o p -- python3 $R/bench.py --steps 40 --warmup 8 $A > $R/$S/tcc_${cfg}_bf16.log 2>&1"
done
exit $STEP_RC
