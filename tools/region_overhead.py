"""Host overhead inside bench.py's timed region (measurement tool): one 20-tick fs_step_n launch of
the C3 workload between two synchronizes, timed on the host clock, with the pieces of Python
around the launch varied.  Prints the median region per variant (microseconds)."""
import ctypes as C
import json
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from footsies_gym_amd import _abi  # noqa: E402
from footsies_gym_amd._lib import lib  # noqa: E402
from footsies_gym_amd.simulator import FootsiesSim  # noqa: E402

N, T, R = 65536, 20, 101
dev = torch.device("cuda", 0)
sim = FootsiesSim(N, device=0, p2_mode="external", seed=0)
h = sim.handle
p1, p2 = sim.hash_actions(R * T + 100, seed=0x5EED)
traj = sim.alloc_trajectory(T)
td = _abi.fs_outputs(**{k: traj[k].data_ptr() for k in _abi.OUTPUT_SPEC})
b1, b2 = p1.data_ptr(), p2.data_ptr()
L = lib()
fs_step_n = L.fs_step_n
torch.cuda.synchronize(dev)


def run(variant):
    walls = []
    for r in range(R):
        k = (r * T) % (R * T)
        a1, a2, tdr = C.c_void_p(b1 + k * N), C.c_void_p(b2 + k * N), C.byref(td)
        if variant in ("dev_sync", "prebuilt_dev_sync"):
            sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731
        else:
            sync = torch.cuda.synchronize
        sync()
        t0 = time.perf_counter()
        if variant.startswith("prebuilt"):
            rc = fs_step_n(h, T, a1, a2, 0, tdr)
        else:
            rc = fs_step_n(h, T, C.c_void_p(b1 + k * N), C.c_void_p(b2 + k * N), 0, C.byref(td))
        sync()
        walls.append(time.perf_counter() - t0)
        assert rc == 0
    walls.sort()
    return round(1e6 * walls[len(walls) // 2], 2)


out = {}
for rep in range(2):
    for v in ("dev_sync", "prebuilt_dev_sync", "sync", "prebuilt_sync"):
        out.setdefault(v, []).append(run(v))
# the synchronize calls alone, nothing launched
for name, sync in (("dev_sync_empty", lambda: torch.cuda.synchronize(dev)), ("sync_empty", torch.cuda.synchronize)):
    w = []
    for _ in range(R):
        sync()
        t0 = time.perf_counter()
        sync()
        w.append(time.perf_counter() - t0)
    w.sort()
    out[name] = round(1e6 * w[len(w) // 2], 2)
print(json.dumps(out))
