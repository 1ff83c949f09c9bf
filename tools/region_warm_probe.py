"""Driver-shape regions right after setup (as bench.py runs them: a 5-tick warm-up, then regions)
vs after a long run of regions: is the first regions' extra time the GPU coming out of idle?"""
import ctypes as C, sys, time
sys.path.insert(0, "/root/repo")
import torch
from footsies_gym_amd import _abi
from footsies_gym_amd._lib import lib
from footsies_gym_amd.simulator import FootsiesSim
N, K, R = 65536, 20, 300
sim = FootsiesSim(N, p2_mode="external", seed=0)
h = sim.handle
p1, p2 = sim.hash_actions(5 + K * R, seed=0x5EED)
traj = sim.alloc_packed_trajectory(K)
td = _abi.fs_packed_traj(lanes=traj["lanes"].data_ptr(), reward=traj["reward"].data_ptr(),
                         final_lanes=traj["final_lanes"].data_ptr())
f = lib().fs_step_n_packed
b1, b2 = p1.data_ptr(), p2.data_ptr()
q1 = [C.c_void_p(b1 + k * N) for k in range(5 + K * R)]
q2 = [C.c_void_p(b2 + k * N) for k in range(5 + K * R)]
tdr = C.byref(td)
torch.cuda.synchronize()
time.sleep(0.5)  # idle, as after the bench's setup
f(h, 5, q1[0], q2[0], tdr)  # the driver's --warmup 5
torch.cuda.synchronize()
walls = []
for r in range(R):
    k = 5 + r * K
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    f(h, K, q1[k], q2[k], tdr)
    torch.cuda.synchronize()
    walls.append(time.perf_counter() - t0)
us = [round(1e6 * w, 1) for w in walls]
print("first 10 regions (us):", us[:10])
for lo, hi in ((0, 5), (5, 20), (20, 50), (50, 100), (100, 300)):
    v = sorted(us[lo:hi])
    print("regions %3d-%3d median %.1f us" % (lo, hi, v[len(v) // 2]))
