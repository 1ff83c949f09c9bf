#!/usr/bin/env python3
"""Where the wall time of a short timed region goes.

The driver runs `bench.py --steps 20 --warmup 5`: one 20-tick fs_step_n launch inside
barrier + synchronize brackets.  This probe times the pieces of that region separately
at the C3 size: an idle synchronize, an empty event-bracketed region, the host side of
the fs_step_n call, and the whole region, each repeated so the medians are stable.

    python tools/region_probe.py [--envs 65536] [--ticks 20] [--reps 50]
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--ticks", type=int, default=20)
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    import torch

    from footsies_gym_amd import _abi
    from footsies_gym_amd._lib import lib
    from footsies_gym_amd.simulator import FootsiesSim

    N, T, R = args.envs, args.ticks, args.reps
    dev = torch.device("cuda", 0)
    sim = FootsiesSim(N, device=0, p2_mode="external", seed=0)
    h = sim.handle
    p1, p2 = sim.hash_actions(T * (R + 2), seed=0x5EED, t0=0)
    traj = sim.alloc_trajectory(T)
    td = _abi.fs_outputs(**{k: traj[k].data_ptr() for k in _abi.OUTPUT_SPEC})
    b1, b2 = p1.data_ptr(), p2.data_ptr()
    L = lib()

    def launch(j):
        return L.fs_step_n(h, T, C.c_void_p(b1 + j * T * N), C.c_void_p(b2 + j * T * N), 0, C.byref(td))

    launch(0)
    torch.cuda.synchronize(dev)
    med = lambda xs: 1e6 * statistics.median(xs)  # noqa: E731
    res = {}

    xs = []
    for _ in range(R):
        t = time.perf_counter()
        torch.cuda.synchronize(dev)
        xs.append(time.perf_counter() - t)
    res["idle_synchronize_us"] = med(xs)

    xs = []
    for _ in range(R):
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t = time.perf_counter()
        e0.record()
        e1.record()
        torch.cuda.synchronize(dev)
        xs.append(time.perf_counter() - t)
    res["empty_event_region_us"] = med(xs)

    host, wall, ev, wall_noev, stream_sync = [], [], [], [], []
    s = torch.cuda.current_stream(dev)
    for j in range(R):
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t = time.perf_counter()
        e0.record()
        t1 = time.perf_counter()
        launch(1 + j % R)
        host.append(time.perf_counter() - t1)
        e1.record()
        torch.cuda.synchronize(dev)
        wall.append(time.perf_counter() - t)
        ev.append(e0.elapsed_time(e1) / 1e3)
    for j in range(R):
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        launch(1 + j % R)
        torch.cuda.synchronize(dev)
        wall_noev.append(time.perf_counter() - t)
    for j in range(R):
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        launch(1 + j % R)
        s.synchronize()
        stream_sync.append(time.perf_counter() - t)
    res.update({"fs_step_n_host_call_us": med(host), "region_wall_us": med(wall), "region_event_us": med(ev),
                "region_wall_no_events_us": med(wall_noev), "region_wall_stream_sync_us": med(stream_sync)})
    # the same ticks in back-to-back launches (queue kept full): the kernel alone
    torch.cuda.synchronize(dev)
    torch.cuda._sleep(int(2e7))
    pairs = []
    for j in range(R):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        launch(1 + j % R)
        e1.record()
        pairs.append((e0, e1))
    torch.cuda.synchronize(dev)
    res["kernel_back_to_back_us"] = 1e6 * statistics.median(a.elapsed_time(b) / 1e3 for a, b in pairs)
    res.update({"envs": N, "ticks": T, "reps": R})
    print(json.dumps(res))
    sim.close()


if __name__ == "__main__":
    main()
