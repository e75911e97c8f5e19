"""The replay sample/gather leg of bench.py alone (for rocprofv3 kernel-trace
and PMC passes of replay_gather_kernel): a full 1e6-row C2 buffer, then the
sweep of bench.gather_sweep.  Prints the sweep as JSON.

    python tools/gather_bench.py [reps] [B ...]
"""
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "soft-actor-critic_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from sac.replay_buffer import ReplayBuffer  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
c = bench.CONFIGS["c2"]
rb = ReplayBuffer(c["capacity"], device=dev, obs_dim=c["obs"], act_dim=c["act"],
                  layout=os.environ.get("REPLAY_LAYOUT", "records"))
bench.synthetic_replay(rb, c["capacity"], c["obs"], c["act"], 0)
sizes = tuple(int(x) for x in sys.argv[2:]) or (256, 4096, 65536, 1_048_576)
print(json.dumps(bench.gather_sweep(rb, dev, sizes=sizes, reps=reps)), flush=True)
