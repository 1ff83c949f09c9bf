"""Driver-shape region (sync, one 20-tick fs_step_n_packed launch, sync) with the launch's ctypes
arguments built in the loop (bench.py today) vs built before the region; interleaved."""
import ctypes as C, sys, time
sys.path.insert(0, "/root/repo")
import torch
from footsies_gym_amd import _abi
from footsies_gym_amd._lib import lib
from footsies_gym_amd.simulator import FootsiesSim
N, K, R = 65536, 20, 400
sim = FootsiesSim(N, p2_mode="external", seed=0)
h = sim.handle
p1, p2 = sim.hash_actions(K * (R + 1), seed=0x5EED)
traj = sim.alloc_packed_trajectory(K)
td = _abi.fs_packed_traj(lanes=traj["lanes"].data_ptr(), reward=traj["reward"].data_ptr(),
                         final_lanes=traj["final_lanes"].data_ptr())
L = lib(); f = L.fs_step_n_packed
b1, b2 = p1.data_ptr(), p2.data_ptr()
pre = [(C.c_void_p(b1 + k * N), C.c_void_p(b2 + k * N)) for k in range(0, K * (R + 1), K)]
tdr = C.byref(td)
f(h, K, pre[0][0], pre[0][1], tdr); torch.cuda.synchronize()
res = {"inline": [], "prebuilt": []}
for r in range(R):
    for mode in ("inline", "prebuilt"):
        k = (r % R) * K
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if mode == "inline":
            f(h, K, C.c_void_p(b1 + k * N), C.c_void_p(b2 + k * N), C.byref(td))
        else:
            a, b = pre[r % R]
            f(h, K, a, b, tdr)
        torch.cuda.synchronize()
        res[mode].append(time.perf_counter() - t0)
for m, v in res.items():
    v.sort()
    print(m, "median %.2f us  p10 %.2f  p90 %.2f" % (1e6 * v[len(v) // 2], 1e6 * v[len(v) // 10], 1e6 * v[9 * len(v) // 10]))
