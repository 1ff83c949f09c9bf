"""bench.py's vector_env leg alone, twice in one process, with the numpy env's outputs in pinned host
memory (the default) and in HBM with one copy a step (FOOTSIES_VENV_DEVICE_OUTPUTS=1), optionally
after the PPO leg (--after-ppo) -- to tell the env's own cost from what the legs before it leave
behind in the bench process.  GPU box only."""
import os
import sys
import time

sys.path.insert(0, "/root/repo")
import torch  # noqa: E402

import bench  # noqa: E402
from footsies_gym_amd import vector_env as ve  # noqa: E402

if os.environ.get("FOOTSIES_VENV_DEVICE_OUTPUTS") == "1":
    _init = ve.FootsiesVectorEnv.__init__

    def init(self, *a, **k):
        k.setdefault("_host_outputs", False)
        _init(self, *a, **k)
    ve.FootsiesVectorEnv.__init__ = init

if "--after-ppo" in sys.argv:
    t = time.perf_counter()
    bench.ppo_rate(torch, 65536, 0)
    print("ppo leg %.1f s" % (time.perf_counter() - t), flush=True)
for r in range(2):
    res = bench.vector_env_rate(torch, 65536, 200, 0)
    print("run %d numpy %.4f ms  torch %.4f ms" % (r, res["numpy"]["ms_per_step"], res["torch"]["ms_per_step"]), flush=True)
