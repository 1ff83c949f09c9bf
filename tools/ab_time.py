#!/usr/bin/env python3
"""A/B timing of built libfootsies.so variants on the GPU (measurement only).

  python tools/ab_time.py LIB[@VAR=VALUE,...] [LIB ...] [--rounds R] [--envs N] [--ticks T]

Each library is timed in its own subprocess (FOOTSIES_LIB override), rounds interleaved so
box-level drift hits every variant alike.  Per library and P2 mode (external = C3, bot = C2):
the median duration of back-to-back fs_step_n launches (fs_step_n_packed with --packed, or per
library with @AB_PACKED=1 / 0) of T ticks over N arenas with full trajectories, bracketed by HIP
events on the launch stream.
"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CODE = r'''
import ctypes as C, os, sys, torch
sys.path.insert(0, %(root)r)
from footsies_gym_amd import _abi
from footsies_gym_amd._lib import check, lib
from footsies_gym_amd.simulator import FootsiesSim
N, T, launches = %(envs)d, %(ticks)d, %(launches)d
res = []
for mode in ("external", "bot"):
    sim = FootsiesSim(N, p2_mode=mode, seed=0)
    p1, p2 = sim.hash_actions(T, seed=0x5EED, p2=(mode == "external"))
    q2 = C.c_void_p(p2.data_ptr()) if mode == "external" else None
    if int(os.environ.get("AB_PACKED", %(packed)d)):  # fs_step_n_packed into packed records (the bench's layout)
        traj = sim.alloc_packed_trajectory(T)
        td = _abi.fs_packed_traj(lanes=traj["lanes"].data_ptr(), reward=traj["reward"].data_ptr(),
                                 final_lanes=traj["final_lanes"].data_ptr())
        def run():
            check(lib().fs_step_n_packed(sim.handle, T, C.c_void_p(p1.data_ptr()), q2, C.byref(td)), sim.handle)
    else:
        traj = sim.alloc_trajectory(T)
        td = _abi.fs_outputs(**{k: traj[k].data_ptr() for k in _abi.OUTPUT_SPEC})
        def run():
            check(lib().fs_step_n(sim.handle, T, C.c_void_p(p1.data_ptr()), q2, 0, C.byref(td)), sim.handle)
    run(); torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
    torch.cuda._sleep(int(2e7))
    for a, b in evs:
        a.record(); run(); b.record()
    torch.cuda.synchronize()
    d = sorted(a.elapsed_time(b) * 1e3 for a, b in evs)
    res.append(d[len(d) // 2])
    if mode == "external":  # the host-driven path: fs_step, one launch per tick (VectorEnv.step)
        def one(k):  # action row k mod T: the rows hold T ticks
            k %%= T
            check(lib().fs_step(sim.handle, C.c_void_p(p1.data_ptr() + k * N), q2 if q2 is None else
                                C.c_void_p(p2.data_ptr() + k * N), _abi.FS_ACT_DEVICE), sim.handle)
        for k in range(20):
            one(k)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(2e7))
        e0.record()
        for k in range(300):
            one(k)
        e1.record()
        torch.cuda.synchronize()
        step_us = e0.elapsed_time(e1) * 1e3 / 300
    del traj, p1, p2
    sim.close()
print("RESULT %%.1f %%.1f %%.2f" %% (res[0], res[1], step_us))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--ticks", type=int, default=1000)
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--packed", action="store_true", help="time fs_step_n_packed (the bench's layout)")
    a = ap.parse_args()
    code = CODE % dict(root=ROOT, envs=a.envs, ticks=a.ticks, launches=a.launches, packed=int(a.packed))
    times = {lib: [] for lib in a.libs}
    for r in range(a.rounds):
        for lib in a.libs:
            # LIB[@VAR=VALUE,...]: the same library under a different environment (e.g.
            # FOOTSIES_FUSED_LANES=2 for the two-lane fused kernel)
            path, _, extra = lib.partition("@")
            env = dict(os.environ, FOOTSIES_LIB=os.path.abspath(path))
            env.update(kv.split("=", 1) for kv in extra.split(",") if kv)
            p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
            line = [x for x in p.stdout.splitlines() if x.startswith("RESULT")]
            if p.returncode or not line:
                print("%s: error\n%s" % (lib, p.stderr[-800:]), flush=True)
                sys.exit(1)
            ext, bot, step = (float(x) for x in line[0].split()[1:])
            times[lib].append((ext, bot, step))
            print("round %d %-40s C3 %8.1f us  C2 %8.1f us  fs_step %6.2f us" % (r, lib, ext, bot, step), flush=True)
    base = None
    for lib, ts in times.items():
        ext = sorted(t[0] for t in ts)[len(ts) // 2]
        bot = sorted(t[1] for t in ts)[len(ts) // 2]
        step = sorted(t[2] for t in ts)[len(ts) // 2]
        if base is None:
            base = (ext, bot, step)
        print("%-40s C3 %8.1f us (%.3e env-steps/s, %+.1f%%)  C2 %8.1f us (%.3e, %+.1f%%)  fs_step %.2f us (%+.1f%%)" % (
            lib, ext, a.envs * a.ticks / ext * 1e6, 100 * (base[0] / ext - 1), bot, a.envs * a.ticks / bot * 1e6,
            100 * (base[1] / bot - 1), step, 100 * (base[2] / step - 1)), flush=True)


if __name__ == "__main__":
    main()
