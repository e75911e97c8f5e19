source tools/gpu_steps.sh
R=$PWD
mkdir -p gpurun_out/wprof
step 200 "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/wprof/fp32 -o kt -- python3 $R/bench.py --config c3 --steps 60 --warmup 10 --no-cpu-baseline --no-sweep --no-bf16 > $R/gpurun_out/wprof/fp32.log 2>&1"
step 200 "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/wprof/bf16 -o kt -- python3 $R/bench.py --config c3 --precision bf16 --steps 60 --warmup 10 --no-cpu-baseline --no-sweep --no-bf16 > $R/gpurun_out/wprof/bf16.log 2>&1"
find gpurun_out/wprof -name "*.db" -delete
for p in fp32 bf16; do f=$(find gpurun_out/wprof/$p -name "*kernel_trace.csv" | head -1); python3 tools/wide_trace.py $f > gpurun_out/wprof/trace_$p.txt; done
exit $STEP_RC
