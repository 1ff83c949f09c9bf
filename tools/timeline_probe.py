#!/usr/bin/env python3
"""Where the fixed cost of a short fused launch goes (measurement only).

  python tools/timeline_probe.py build              # exp/timeline/libfootsies.so (CPU, here)
  python tools/timeline_probe.py run [--envs N]     # on the GPU box, with that library

`build` makes a variant of fs_kernels.hip whose step kernels stamp each wave with
s_memrealtime (the 100 MHz constant clock every CU shares) at four points:
  t0 kernel entry, t1 after the prologue (state loads + table staging, the block barrier),
  t2 after the tick loop, t3 after the final state stores have drained (vmcnt(0)),
plus the wave's HW_ID / XCC_ID, written by lane 0 with ordinary vector stores into a
device array the host copies out.  `run` times fs_step_n launches of 1..1000 ticks at
N arenas (back-to-back, HIP events on the launch stream) and reads the stamps of one
isolated launch per shape, so the intercept of launch time vs ticks splits into the
dispatch ramp (spread of t0), the prologue, the per-tick loop and the drain.
The stamped kernel is otherwise the product kernel; its results are not checked here.
"""
import argparse
import ctypes as C
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "runs", "timeline")  # (git-ignored; travels to the GPU box)
NSTAMP = 8  # u64 per wave: t0 t1 t2 t3 hwid xcc pad pad
MAXWAVES = 16384

PRELUDE = r'''
__device__ unsigned long long g_fs_stamps[%d * %d];
extern "C" __attribute__((visibility("default"))) int fs_dbg_stamps(void* dst, size_t bytes) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_fs_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
''' % (MAXWAVES, NSTAMP)


def variant_source():
    with open(os.path.join(ROOT, "footsies_gym_amd", "csrc", "fs_kernels.hip")) as f:
        s = f.read()
    anchor = "#pragma clang fp contract(off)\n"
    assert anchor in s
    s = s.replace(anchor, anchor + PRELUDE, 1)
    a = "  const int l = blockIdx.x * blockDim.x + threadIdx.x;\n  const bool active = l < 2 * p.n_envs;\n"
    assert a in s
    s = s.replace(a, a + "  const uint64_t ts0 = __builtin_amdgcn_s_memrealtime();\n", 1)
    b = "  if constexpr (FUSED) stage_tables<P2 == FS_P2_BOT || P2 == kActors>();\n"
    assert b in s
    s = s.replace(b, b + "  const uint64_t ts1 = __builtin_amdgcn_s_memrealtime();\n", 1)
    c = ("  if (active) {\n    store_lane<P2>(L, p.st, a);\n"
         "    if constexpr (GEOM) reinterpret_cast<float*>(p.st.posy)[2 * a + (int)k] = L.f.y;\n  }\n}\n")
    assert c in s
    s = s.replace(c, (
        "  const uint64_t ts2 = __builtin_amdgcn_s_memrealtime();\n"
        "  if (active) store_lane<P2>(L, p.st, a);\n"
        "  asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n"
        "  const uint64_t ts3 = __builtin_amdgcn_s_memrealtime();\n"
        "  const uint32_t w = (uint32_t)l >> 6;\n"
        "  if ((threadIdx.x & 63) == 0 && w < %du) {\n"
        "    unsigned long long* d = g_fs_stamps + (size_t)w * %d;\n"
        "    d[0] = ts0; d[1] = ts1; d[2] = ts2; d[3] = ts3;\n"
        "    d[4] = (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11));\n"
        "    d[5] = (unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11));\n"
        "  }\n}\n") % (MAXWAVES, NSTAMP), 1)
    return s


def build():
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(OUT, "fs_kernels_timeline.hip")
    with open(src, "w") as f:
        f.write(variant_source())
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "build_variant.py"), src, OUT], check=True)


def run(envs, reps, packed=False):
    os.environ["FOOTSIES_LIB"] = os.path.join(OUT, "libfootsies.so")
    import torch

    from footsies_gym_amd import _abi
    from footsies_gym_amd._lib import check, lib
    from footsies_gym_amd.simulator import FootsiesSim

    N = envs
    L = lib()
    L.fs_dbg_stamps.restype = C.c_int
    L.fs_dbg_stamps.argtypes = [C.c_void_p, C.c_size_t]
    sim = FootsiesSim(N, device=0, p2_mode="external", seed=0)
    h = sim.handle
    tmax = 1000
    p1, p2 = sim.hash_actions(tmax, seed=0x5EED, t0=0)
    if packed:  # the bench's layout (fs_step_n_packed)
        traj = sim.alloc_packed_trajectory(tmax)
        td = _abi.fs_packed_traj(lanes=traj["lanes"].data_ptr(), reward=traj["reward"].data_ptr(),
                                 final_lanes=traj["final_lanes"].data_ptr())
    else:
        traj = sim.alloc_trajectory(tmax)
        td = _abi.fs_outputs(**{k: traj[k].data_ptr() for k in _abi.OUTPUT_SPEC})
    b1, b2 = p1.data_ptr(), p2.data_ptr()
    waves = (2 * N + 63) // 64
    buf = (C.c_uint64 * (waves * NSTAMP))()

    def launch(n):
        if packed:
            check(L.fs_step_n_packed(h, n, C.c_void_p(b1), C.c_void_p(b2), C.byref(td)), h)
        else:
            check(L.fs_step_n(h, n, C.c_void_p(b1), C.c_void_p(b2), 0, C.byref(td)), h)

    # warm the clock and the pages
    for _ in range(3):
        launch(tmax)
    torch.cuda.synchronize()
    res = {"envs": N, "waves": waves, "shapes": []}
    for n in (1, 2, 5, 10, 20, 50, 100, 1000):
        r = reps if n < 1000 else max(3, reps // 10)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(r)]
        torch.cuda._sleep(int(2e7))
        for a, b in evs:
            a.record()
            launch(n)
            b.record()
        torch.cuda.synchronize()
        b2b = statistics.median(a.elapsed_time(b) * 1e3 for a, b in evs)
        # isolated launches: stamps of the last one, walls of all
        launch(tmax)  # keep the clock up
        torch.cuda.synchronize()
        import time
        walls = []
        for _ in range(r):
            torch.cuda.synchronize()
            t = time.perf_counter()
            launch(n)
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t) * 1e6)
        check(L.fs_dbg_stamps(C.cast(buf, C.c_void_p), C.sizeof(buf)))
        st = [tuple(buf[w * NSTAMP + j] for j in range(6)) for w in range(waves)]
        t0 = min(s[0] for s in st)
        us = lambda v: (v - t0) / 100.0  # noqa: E731  100 MHz -> us
        starts = sorted(us(s[0]) for s in st)
        pro = sorted((s[1] - s[0]) / 100.0 for s in st)
        loop = sorted((s[2] - s[1]) / 100.0 for s in st)
        drain = sorted((s[3] - s[2]) / 100.0 for s in st)
        ends = sorted(us(s[3]) for s in st)
        q = lambda xs, f: xs[min(len(xs) - 1, int(f * len(xs)))]  # noqa: E731
        xcc = {}
        for s in st:
            xcc.setdefault(int(s[5]) & 0xF, []).append(us(s[0]))
        # the waves sharing a SIMD (HW_ID: wave slot 3:0, SIMD 5:4, CU 11:8, SH 12, SE 15:13 -- with the XCC):
        # how far apart their loops end, and how long the last one runs alone
        simd = {}
        for s in st:
            hw = int(s[4])
            simd.setdefault((int(s[5]) & 0xF, (hw >> 13) & 7, (hw >> 8) & 31, (hw >> 4) & 3), []).append(s)
        gaps = sorted((max(x[2] for x in g) - min(x[2] for x in g)) / 100.0 for g in simd.values() if len(g) > 1)
        res["shapes"].append({
            "ticks": n, "b2b_us": round(b2b, 2), "isolated_wall_us": round(statistics.median(walls), 2),
            "wave_start_us": {"p0": 0.0, "p50": round(q(starts, .5), 2), "p90": round(q(starts, .9), 2),
                              "max": round(starts[-1], 2)},
            "prologue_us": {"p10": round(q(pro, .1), 2), "p50": round(q(pro, .5), 2), "max": round(pro[-1], 2)},
            "loop_us": {"p10": round(q(loop, .1), 2), "p50": round(q(loop, .5), 2), "max": round(loop[-1], 2)},
            "loop_us_per_tick_p50": round(q(loop, .5) / n, 4),
            "drain_us": {"p50": round(q(drain, .5), 2), "max": round(drain[-1], 2)},
            "wave_end_us": {"p50": round(q(ends, .5), 2), "max": round(ends[-1], 2)},
            "simd_pair_loop_end_gap_us": {"p50": round(q(gaps, .5), 2), "p90": round(q(gaps, .9), 2),
                                          "max": round(gaps[-1], 2)} if gaps else None,
            "first_start_by_xcc_us": {str(k): round(min(v), 2) for k, v in sorted(xcc.items())},
            "last_start_by_xcc_us": {str(k): round(max(v), 2) for k, v in sorted(xcc.items())},
        })
        print(json.dumps(res["shapes"][-1]), flush=True)
        if n in (20, 1000):
            res["raw_%d" % n] = [[int(v) for v in s_] for s_ in st]
    sim.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "timeline.json"))
    ap.add_argument("--packed", action="store_true", help="fs_step_n_packed launches (the bench's layout)")
    a = ap.parse_args()
    if a.cmd == "build":
        build()
        return
    res = run(a.envs, a.reps, a.packed)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
