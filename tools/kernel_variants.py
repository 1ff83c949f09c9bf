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


ENV_STEP = "__device__ __forceinline__ void env_step(Lane& L, uint32_t a_own"
VNOP100 = "  asm volatile(\"" + "v_nop\\n" * 100 + "\");"
LDS2 = ("  { uint32_t d0; asm volatile(\"ds_read_b32 %0, %1\\n s_waitcnt lgkmcnt(0)\\n v_and_b32 %0, 0xfc, %0\\n "
        "ds_read_b32 %0, %0\\n s_waitcnt lgkmcnt(0)\" : \"=v\"(d0) : \"v\"((uint32_t)0)); (void)d0; }")
SALU50 = "  { uint32_t s0 = 0; asm volatile(\"" + "s_add_u32 %0, %0, 1\\n" * 50 + "\" : \"+s\"(s0)); }"

VADD100_IND = ("  { uint32_t r0 = 1, r1 = 2, r2 = 3, r3 = 4; asm volatile(\"" +
               "v_add_u32 %0, 1, %0\\n v_add_u32 %1, 1, %1\\n v_add_u32 %2, 1, %2\\n v_add_u32 %3, 1, %3\\n" * 25 +
               "\" : \"+v\"(r0), \"+v\"(r1), \"+v\"(r2), \"+v\"(r3)); }")
VADD100_DEP = "  { uint32_t r0 = 1; asm volatile(\"" + "v_add_u32 %0, 1, %0\\n" * 100 + "\" : \"+v\"(r0)); }"
VOP3_100 = ("  { uint32_t r0 = 1, r1 = 2, r2 = 3, r3 = 4; asm volatile(\"" +
            "v_add3_u32 %0, %0, 1, %1\\n v_add3_u32 %1, %1, 1, %2\\n v_add3_u32 %2, %2, 1, %3\\n "
            "v_add3_u32 %3, %3, 1, %0\\n" * 25 + "\" : \"+v\"(r0), \"+v\"(r1), \"+v\"(r2), \"+v\"(r3)); }")

VARIANTS = {
    "base": lambda s: s,
    "block512": lambda s: s.replace("constexpr int kBlock = 256;", "constexpr int kBlock = 512;").replace(
        "__launch_bounds__(256)", "__launch_bounds__(512)"),
    "plus_100_vadd_ind": lambda s: _edit_fn(s, ENV_STEP, VADD100_IND),
    "plus_100_vadd_dep": lambda s: _edit_fn(s, ENV_STEP, VADD100_DEP),
    "plus_100_vop3": lambda s: _edit_fn(s, ENV_STEP, VOP3_100),
    "plus_100_valu": lambda s: _edit_fn(s, ENV_STEP, VNOP100),
    "plus_2_lds_rt": lambda s: _edit_fn(s, ENV_STEP, LDS2),
    "plus_50_salu": lambda s: _edit_fn(s, ENV_STEP, SALU50),
    "no_stores": lambda s: _edit_fn(_edit_fn(s, "__device__ __forceinline__ void write_obs(", "  return;"),
                                    "__device__ __forceinline__ void env_step(Lane& L, uint32_t a_own",
                                    "  const_cast<StepParams&>(p).dense_reward = p.dense_reward;"
                                    ).replace("    o.reward[r] = reward;\n", "").replace(
                                        "    o.terminated[r] = over ? 1 : 0;\n", "").replace(
                                        "    o.truncated[r] = 0;\n", ""),
    "_const_actions": lambda s: s.replace(
        "    else return src[(uint32_t)t * (uint32_t)p.n_envs + (uint32_t)a];",
        "    else return (uint32_t)(t * 5 + a) & 7u;"),
    "_no_collision": lambda s: _edit_fn(s, "__device__ __forceinline__ void hitbox_hurtbox_collision(", "  return;"),
    "_no_push": lambda s: _edit_fn(s, "__device__ __forceinline__ void push_character_vs_character(", "  return;"),
    "_no_request": lambda s: _edit_fn(s, "__device__ __forceinline__ void update_action_request(", "  return;"),
}


def active():
    """Variants whose name starts with "_" change the game's dynamics (removed phases alter
    what the arenas do), so their times are not comparable; they are kept but not run."""
    return {k: v for k, v in VARIANTS.items() if not k.startswith("_")}


def build():
    sys.path.insert(0, ROOT)
    from footsies_gym_amd import build as B
    for name, fn in active().items():
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
            subprocess.run([B._hipcc(), "--offload-arch=gfx950", *B.flags_for(s), "-I", os.path.join(ROOT, "include"),
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
    for name in active():
        print("%-14s median us per 100-tick launch: %s" % (name, time_one(os.path.join(EXP, name, "libfootsies.so"),
                                                                          N, T)), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        time_all(*(int(x) for x in sys.argv[2:]))
