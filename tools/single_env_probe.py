"""Where a one-arena step's time goes (measurement tool): per-step host wall of fs_step with
host actions (FS_ACT_HOST: pinned staging + H2D copy) or device actions, each followed by
fs_sync, by outputs_numpy's D2H copy, or by the whole FootsiesEnv.step.  Median of 2000 steps."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from footsies_gym_amd import _abi  # noqa: E402
from footsies_gym_amd._lib import lib  # noqa: E402
from footsies_gym_amd.simulator import FootsiesSim  # noqa: E402
from footsies_gym_amd.vector_env import FootsiesEnv  # noqa: E402

R = 2000
L = lib()


def med(fn):
    for _ in range(100):
        fn()
    w = []
    for _ in range(R):
        t = time.perf_counter()
        fn()
        w.append(time.perf_counter() - t)
    w.sort()
    return round(1e6 * w[R // 2], 2)


sim = FootsiesSim(1, device=0, p2_mode="bot", seed=0)
h = sim.handle
ha = np.zeros(1, np.uint8)
da = torch.zeros(1, dtype=torch.uint8, device="cuda")
out = {}
out["host_actions_sync"] = med(lambda: (L.fs_step(h, ha.ctypes.data, None, _abi.FS_ACT_HOST), L.fs_sync(h)))
out["device_actions_sync"] = med(lambda: (L.fs_step(h, da.data_ptr(), None, _abi.FS_ACT_DEVICE), L.fs_sync(h)))
out["device_actions_d2h"] = med(lambda: (L.fs_step(h, da.data_ptr(), None, _abi.FS_ACT_DEVICE), sim.outputs_numpy(copy=False)))
out["host_actions_d2h"] = med(lambda: (L.fs_step(h, ha.ctypes.data, None, _abi.FS_ACT_HOST), sim.outputs_numpy(copy=False)))
out["sim_step_numpy_d2h"] = med(lambda: (sim.step(np.zeros((1, 3), bool)), sim.outputs_numpy(copy=False)))
out["sync_only"] = med(lambda: L.fs_sync(h))
sim.close()
env = FootsiesEnv(seed=0)
env.reset()
a = (False, True, False)


def st():
    if env.step(a)[2]:
        env.reset()
out["footsies_env_step"] = med(st)
env.close()
print(json.dumps(out))
