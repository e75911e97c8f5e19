# Round-5 check of the current build on the GPU box: the GPU suite (tie-free
# parity draws print their redraw counts: -s), smoke, the default bench line,
# then (R05_PROF=1) rocprofv3 kernel stats + FETCH / WRITE / TCC hit-miss
# passes for the bf16 C2 and C3 steps, condensed on the
# box into small files; the databases are removed (gpurun_out <= 64 MiB).
source tools/gpu_steps.sh
R=${GRAFT_REPO_ROOT:-$PWD}
S=$R/gpurun_out/${R05_OUT:-r05_check}
mkdir -p $S
if [ -z "${R05_ONLY_PROF:-}" ]; then
step 900 "python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $S/gputest.log 2>&1"
step 200 "python -c 'import __graft_entry__ as g; g.smoke()' > $S/smoke.log 2>&1"
step 400 "python bench.py > $S/bench.json 2> $S/bench.err"
fi
if [ -n "${R05_PROF:-}" ]; then
cd /tmp && export TMPDIR=/tmp
for cp in ${R05_PROF_SET:-c2:bf16 c3:bf16}; do
  cfg=${cp%%:*}; prec=${cp##*:}
  P=$S/prof_${cfg}_${prec}
  A="--config $cfg --precision $prec --no-cpu-baseline --no-sweep --no-bf16 --no-c3"
  step 200 "rocprofv3 --kernel-trace --stats -d $P/kt -o kt -- python3 $R/bench.py --steps 400 --warmup 50 $A > $S/kt_${cfg}_${prec}.log 2>&1"
  step 120 "rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o p -- python3 $R/bench.py --steps 40 --warmup 8 $A > $S/fetch_${cfg}_${prec}.log 2>&1"
  step 120 "rocprofv3 --pmc WRITE_SIZE -d $P/write -o p -- python3 $R/bench.py --steps 40 --warmup 8 $A > $S/write_${cfg}_${prec}.log 2>&1"
  step 120 "rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $P/tcc -o p -- python3 $R/bench.py --steps 40 --warmup 8 $A > $S/tcc_${cfg}_${prec}.log 2>&1"
  step 60 "python3 $R/tools/pmc_summary.py ${R05_ROUND:-r05} $P --tag _${cfg}_${prec} --config $cfg --precision $prec --dst $S > /dev/null"
  step 60 "python3 $R/tools/pmc_read.py $P/tcc > $S/${R05_ROUND:-r05}_tcc_${cfg}_${prec}.txt"
  rm -rf $P
done
if [ -n "${R05_GATHER:-}" ]; then  # the gather leg's roofline traffic (bench roofline_gather.traffic)
  P=$S/prof_gather
  step 200 "rocprofv3 --kernel-trace --stats -d $P/kt -o kt -- python3 $R/tools/gather_bench.py 20 1048576 > $S/kt_gather.log 2>&1"
  step 200 "rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o p -- python3 $R/tools/gather_bench.py 5 1048576 > $S/fetch_gather.log 2>&1"
  step 200 "rocprofv3 --pmc WRITE_SIZE -d $P/write -o p -- python3 $R/tools/gather_bench.py 5 1048576 > $S/write_gather.log 2>&1"
  step 60 "python3 $R/tools/pmc_summary.py ${R05_ROUND:-r05} $P --tag _gather --config gather --precision fp32 --dst $S > /dev/null"
  rm -rf $P
fi
fi
exit $STEP_RC
