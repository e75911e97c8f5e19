for lib in libsac_engine.so libsac_engine_prev.so libsac_engine.so libsac_engine_prev.so; do
  SAC_ENGINE_LIB=$PWD/soft-actor-critic_amd/$lib timeout -k 10 200 python3 bench.py --steps 200 --warmup 50 --no-cpu-baseline --no-bf16 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('$lib', d['value'], d['replay_gather_GBps_sweep'], d['replay_sample_GBps_sweep'], d['replay_gather_GBps_sweep_soa_layout'])"
done
