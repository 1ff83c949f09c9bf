"""The driver-shaped bench region in a fresh process (measurement tool): 5 warm-up ticks, then 5
regions of one 20-tick fs_step_n launch between synchronizes, optionally after a GPU spin
(torch.cuda._sleep) and / or a host spin, to see whether the first regions pay a cold start;
or after many launches: 3000 one-element torch kernels (torch_launches) or 3000 one-tick
fs_step_n launches (sim_launches) on the same stream.
Usage on the GPU box: python tools/cold_region_probe.py none|gpu_spin|host_spin|both|torch_launches|sim_launches"""
import ctypes as C, json, sys, time, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from footsies_gym_amd import _abi
from footsies_gym_amd._lib import lib
from footsies_gym_amd.simulator import FootsiesSim
variant = sys.argv[1]
N, T, W, R = 65536, 20, 5, 5
dev = torch.device("cuda", 0)
sim = FootsiesSim(N, device=0, p2_mode="external", seed=0)
h = sim.handle
p1, p2 = sim.hash_actions(W + R * T, seed=0x5EED)
traj = sim.alloc_trajectory(T)
td = _abi.fs_outputs(**{k: traj[k].data_ptr() for k in _abi.OUTPUT_SPEC})
b1, b2 = p1.data_ptr(), p2.data_ptr()
fs_step_n = lib().fs_step_n
torch.cuda.synchronize(dev)
assert fs_step_n(h, W, C.c_void_p(b1), C.c_void_p(b2), 0, C.byref(td)) == 0
torch.cuda.synchronize(dev)
if variant in ("gpu_spin", "both"):
    torch.cuda._sleep(int(2e8))  # ~0.1 s of GPU spin
    torch.cuda.synchronize(dev)
if variant in ("host_spin", "both"):
    t = time.perf_counter()
    while time.perf_counter() - t < 0.05:
        pass
if variant == "torch_launches":
    x = torch.zeros(1, device=dev)
    for _ in range(3000):
        x.add_(1)
    torch.cuda.synchronize(dev)
if variant == "sim_launches":
    for j in range(3000):
        assert fs_step_n(h, 1, C.c_void_p(b1 + (j % T) * N), C.c_void_p(b2 + (j % T) * N), 0, C.byref(td)) == 0
    torch.cuda.synchronize(dev)
walls = []
for r in range(R):
    k = W + r * T
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    assert fs_step_n(h, T, C.c_void_p(b1 + k * N), C.c_void_p(b2 + k * N), 0, C.byref(td)) == 0
    torch.cuda.synchronize(dev)
    walls.append(round(1e6 * (time.perf_counter() - t0), 1))
print(json.dumps({"variant": variant, "walls_us": walls, "median": sorted(walls)[R // 2]}))
