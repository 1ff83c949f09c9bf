#!/usr/bin/env python3
"""Ablation builds of the step kernel (measurement only, never shipped).

  python tools/kernel_variants.py build          # exp/<variant>/libfootsies.so
  python tools/kernel_variants.py time [N] [T]   # on the GPU: per-launch time of each

Each variant is a text edit of a copy of fs_kernels.hip that removes one phase of the
tick, so the time it saves bounds what that phase costs.  Results are invalid
simulations by construction.
"""
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "footsies_gym_amd", "csrc")
EXP = os.path.join(ROOT, "exp")


def _edit_fn(src, signature_start, body_prefix):
    """Insert body_prefix right after the opening brace of the function whose definition
    line contains signature_start."""
    i = src.index(signature_start)
    j = src.index("{", i)
    return src[:j + 1] + "\n" + body_prefix + src[j + 1:]


VARIANTS = {
    "base": lambda s: s,
    "no_stores": lambda s: _edit_fn(_edit_fn(s, "__device__ __forceinline__ void write_obs(", "  return;"),
                                    "__device__ __forceinline__ void env_step(Lane& L, uint32_t a_own",
                                    "  const_cast<StepParams&>(p).dense_reward = p.dense_reward;"
                                    ).replace("    o.reward[r] = reward;\n", "").replace(
                                        "    o.terminated[r] = over ? 1 : 0;\n", "").replace(
                                        "    o.truncated[r] = 0;\n", ""),
    "const_actions": lambda s: s.replace(
        "    else return src[(uint32_t)t * (uint32_t)p.n_envs + (uint32_t)a];",
        "    else return (uint32_t)(t * 5 + a) & 7u;"),
    "no_collision": lambda s: _edit_fn(s, "__device__ __forceinline__ void hitbox_hurtbox_collision(", "  return;"),
    "no_push": lambda s: _edit_fn(s, "__device__ __forceinline__ void push_character_vs_character(", "  return;"),
    "no_request": lambda s: _edit_fn(s, "__device__ __forceinline__ void update_action_request(", "  return;"),
}


def build():
    sys.path.insert(0, ROOT)
    from footsies_gym_amd import build as B
    for name, fn in VARIANTS.items():
        d = os.path.join(EXP, name)
        os.makedirs(d, exist_ok=True)
        for f in os.listdir(CSRC):
            if f.endswith((".hip", ".cpp", ".h")):
                shutil.copy(os.path.join(CSRC, f), d)
        src = open(os.path.join(CSRC, "fs_kernels.hip")).read()
        out = fn(src)
        assert name == "base" or out != src, name
        open(os.path.join(d, "fs_kernels.hip"), "w").write(out.replace('#include "fs_internal.h"', '#include "fs_internal.h"'))
        objs = []
        for s in B.SOURCES:
            o = os.path.join(d, s + ".o")
            subprocess.run([B._hipcc(), "--offload-arch=gfx950", *B.CFLAGS, "-I", os.path.join(ROOT, "include"),
                            "-I", CSRC, "-c", os.path.join(d, s), "-o", o], check=True)
            objs.append(o)
        subprocess.run([B._hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                        os.path.join(d, "libfootsies.so"), *objs], check=True)
        for o in objs:
            os.remove(o)
        print("built", name)


def time_one(lib, N, T, chunk=100):
    code = r'''
import ctypes as C, os, sys, torch
sys.path.insert(0, %r)
from footsies_gym_amd import _abi
from footsies_gym_amd._lib import check, lib
from footsies_gym_amd.simulator import FootsiesSim
N, T, chunk = %d, %d, %d
sim = FootsiesSim(N, p2_mode="external")
p1, p2 = sim.hash_actions(T, seed=0x5EED)
traj = sim.alloc_trajectory(chunk)
td = _abi.fs_outputs(**{k: traj[k].data_ptr() for k in _abi.OUTPUT_SPEC})
def run(k0):
    check(lib().fs_step_n(sim.handle, chunk, C.c_void_p(p1.data_ptr() + k0 * N), C.c_void_p(p2.data_ptr() + k0 * N), 0, C.byref(td)), sim.handle)
run(0); torch.cuda.synchronize()
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(T // chunk)]
torch.cuda._sleep(int(2e7))
for j, (a, b) in enumerate(evs):
    a.record(); run(j * chunk); b.record()
torch.cuda.synchronize()
d = sorted(a.elapsed_time(b) * 1e3 for a, b in evs)
print("%%.1f" %% d[len(d) // 2])
''' % (ROOT, N, T, chunk)
    env = dict(os.environ, FOOTSIES_LIB=lib)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    if r.returncode:
        return "error: " + r.stderr[-300:]
    return r.stdout.strip().splitlines()[-1]


def time_all(N=65536, T=2000):
    for name in VARIANTS:
        print("%-14s median us per 100-tick launch: %s" % (name, time_one(os.path.join(EXP, name, "libfootsies.so"),
                                                                          N, T)), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        time_all(*(int(x) for x in sys.argv[2:]))
