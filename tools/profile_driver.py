"""Fixed workload for rocprofv3 runs: W warm-up + R profiled launches of one kernel config.

  python tools/profile_driver.py --mode fused --chunk 100 --launches 5
  python tools/profile_driver.py --mode step --launches 200
  python tools/profile_driver.py --mode fused --layout packed --chunk 1000 --launches 3
"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--mode", choices=["fused", "step"], default="fused")
    ap.add_argument("--chunk", type=int, default=100)
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--p2", default="external")
    ap.add_argument("--layout", choices=["fields", "packed"], default="fields",
                    help="fused mode's trajectory: one array per field (fs_step_n) or packed (fs_step_n_packed)")
    a = ap.parse_args()
    import torch
    from footsies_gym_amd import _abi
    from footsies_gym_amd._lib import check, lib
    from footsies_gym_amd.simulator import FootsiesSim
    N = a.envs
    sim = FootsiesSim(N, p2_mode=a.p2)
    ticks = a.chunk if a.mode == "fused" else 1
    total = ticks * (a.launches + 2)
    p1, p2 = sim.hash_actions(total, seed=0x5EED)
    packed = a.mode == "fused" and a.layout == "packed"
    traj = sim.alloc_packed_trajectory(ticks) if packed else sim.alloc_trajectory(ticks)
    if packed:
        td = _abi.fs_packed_traj(lanes=traj["lanes"].data_ptr(), reward=traj["reward"].data_ptr(),
                                 final_lanes=traj["final_lanes"].data_ptr())
    else:
        td = _abi.fs_outputs(**{k: traj[k].data_ptr() for k in _abi.OUTPUT_SPEC})
    h, L = sim.handle, lib()
    for j in range(a.launches + 2):
        k = j * ticks
        q1 = C.c_void_p(p1.data_ptr() + k * N)
        q2 = C.c_void_p(p2.data_ptr() + k * N) if a.p2 == "external" else None
        if packed:
            check(L.fs_step_n_packed(h, ticks, q1, q2, C.byref(td)), h)
        elif a.mode == "fused":
            check(L.fs_step_n(h, ticks, q1, q2, 0, C.byref(td)), h)
        else:
            check(L.fs_step(h, q1, q2, _abi.FS_ACT_DEVICE), h)
    torch.cuda.synchronize()
    print("ok", a.mode, a.launches + 2, "launches of", ticks, "ticks")


if __name__ == "__main__":
    main()
