"""MI355X-native SAC update engine with the API of ignaschuemer7/soft-actor-critic.

Modules (reference counterparts in parentheses):
    sac.agent          SAC agent, fused HIP training_step   (sac/agent.py)
    sac.models         QNetwork, PolicyNetwork, build_mlp   (sac/models.py)
    sac.replay_buffer  HBM struct-of-arrays ReplayBuffer    (sac/replay_buffer.py)
    sac.envs           probe environments                   (sac/envs.py)
    sac.engine         host wrapper of libsac_engine.so (C ABI: include/sac_engine.h)
    sac.replicas       independent-seed replicas, one process per GPU
"""
__version__ = "0.1.0"
