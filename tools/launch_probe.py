#!/usr/bin/env python3
"""Host-side latency around one short fused launch (measurement only).

  python tools/launch_probe.py [--envs 65536] [--ticks 20] [--reps 60]

Runs the same region -- synchronize, one fs_step_n launch of `ticks` ticks, synchronize,
host wall clock -- in child processes that differ only in how the host waits and which stream
the handle issues on, so the share of the driver-shape region that is not kernel time can be
attributed:
  default      : torch's current (default) stream, torch.cuda.synchronize()
  side_stream  : the handle on a torch.cuda.Stream() of its own, torch.cuda.synchronize()
  no_interrupt : default stream, HSA_ENABLE_INTERRUPT=0 (completion signals polled, not waited
                 on by interrupt) -- set before the runtime starts
Each child also reports the kernel's back-to-back duration (HIP events, queue pre-filled), an
empty region (synchronize; synchronize) and the host time of the fs_step_n call itself.
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import ctypes as C, json, statistics, sys, time
sys.path.insert(0, %(root)r)
import torch
from footsies_gym_amd import _abi
from footsies_gym_amd._lib import lib
from footsies_gym_amd.simulator import FootsiesSim
N, T, R, side = %(envs)d, %(ticks)d, %(reps)d, %(side)d
dev = torch.device("cuda", 0)
sim = FootsiesSim(N, device=0, p2_mode="external", seed=0)
if side:
    sim.use_torch_stream(torch.cuda.Stream(dev))
h = sim.handle
p1, p2 = sim.hash_actions(T * (R + 2), seed=0x5EED, t0=0)
traj = sim.alloc_trajectory(T)
td = _abi.fs_outputs(**{k: traj[k].data_ptr() for k in _abi.OUTPUT_SPEC})
b1, b2 = p1.data_ptr(), p2.data_ptr()
L = lib()
fs_step_n = L.fs_step_n
def launch(j):
    return fs_step_n(h, T, C.c_void_p(b1 + j * T * N), C.c_void_p(b2 + j * T * N), 0, C.byref(td))
for j in range(30):
    launch(j %% R)
torch.cuda.synchronize(dev)
res = {}
xs = []
for _ in range(R):
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    torch.cuda.synchronize(dev)
    xs.append(time.perf_counter() - t)
res["empty_region_us"] = 1e6 * statistics.median(xs)
walls, host = [], []
for j in range(R):
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    launch(j)
    t1 = time.perf_counter()
    torch.cuda.synchronize(dev)
    walls.append(time.perf_counter() - t)
    host.append(t1 - t)
res["region_us"] = 1e6 * statistics.median(walls)
res["region_us_min"] = 1e6 * min(walls)
res["host_call_us"] = 1e6 * statistics.median(host)
abi = L.fs_abi_version
xs = []
for _ in range(R):
    t = time.perf_counter()
    abi()
    xs.append(time.perf_counter() - t)
res["ctypes_trivial_call_us"] = 1e6 * statistics.median(xs)
s = sim.stream
torch.cuda.synchronize(dev)
with torch.cuda.stream(s):
    torch.cuda._sleep(int(2e7))
pairs = []
for j in range(R):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    launch(j)
    e1.record(s)
    pairs.append((e0, e1))
torch.cuda.synchronize(dev)
res["kernel_b2b_us"] = 1e3 * statistics.median(a.elapsed_time(b) for a, b in pairs)
print("RESULT " + json.dumps(res))
sim.close()
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--ticks", type=int, default=20)
    ap.add_argument("--reps", type=int, default=60)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "launch_probe.json"))
    a = ap.parse_args()
    cases = {"default": ({}, 0), "side_stream": ({}, 1), "no_interrupt": ({"HSA_ENABLE_INTERRUPT": "0"}, 0),
             "no_interrupt_side": ({"HSA_ENABLE_INTERRUPT": "0"}, 1),
             "dev_kernarg": ({"HIP_FORCE_DEV_KERNARG": "1"}, 0),
             "host_kernarg": ({"HIP_FORCE_DEV_KERNARG": "0"}, 0)}
    out = {"envs": a.envs, "ticks": a.ticks, "reps": a.reps, "cases": {}}
    for r in range(a.rounds):
        for name, (env, side) in cases.items():
            code = CHILD % dict(root=ROOT, envs=a.envs, ticks=a.ticks, reps=a.reps, side=side)
            p = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), capture_output=True,
                               text=True, timeout=300)
            line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")]
            if p.returncode or not line:
                print(name, "failed", p.stderr[-1500:], flush=True)
                sys.exit(1)
            res = json.loads(line[0][7:])
            out["cases"].setdefault(name, []).append(res)
            print(r, name, json.dumps(res), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
