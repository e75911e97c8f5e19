source tools/gpu_steps.sh
step 200 'DBG_FLIP=1 python -u tools/debug/pi0_grad.py 24 4 512,512 384 2 > gpurun_out/r04_dbg_pi0_512.txt 2>&1'
true
exit $STEP_RC
