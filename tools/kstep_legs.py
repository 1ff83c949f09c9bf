#!/usr/bin/env python3
"""`k_step` (the one-tick launch behind fs_step / FootsiesVectorEnv.step) split by the bench leg
that launched it (one rocprofv3 summary mixed every leg's dispatches).

Run on the GPU box under the kernel trace, then reduce in the build container:

  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kstep -o run -- python3 tools/kstep_legs.py
  python3 tools/kstep_legs.py --reduce gpurun_out/kstep --json profiles/r05_kstep_legs.json

The run drives the same calls bench.py's legs make (65 536 arenas, P2 external unless noted), one
leg after the other, each preceded by a marker dispatch (torch.cuda._sleep, rocprofv3 names it
`spin_kernel`): the reduction assigns every k_step dispatch to the leg whose marker precedes it and
reports per leg the dispatch count and the average / median / min / max / p99 duration, plus the
launch-to-launch period (start of one dispatch to the start of the next, within the leg).
The `venv_torch_policy` leg produces each step's actions on the device just before the step (a
policy's sampling), where the other legs read rows written long before (from HBM).
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# in marker order; the "warm_*" sections (warm-ups between the timed legs) are traced but not reported
LEGS = ["step", "step_warm_first", "host_actions", "step_gather", "step_rec", "warm_venv_torch", "venv_torch", "warm_venv_numpy",
        "venv_numpy", "warm_venv_policy", "venv_torch_policy", "warm_single_env", "single_env"]


def run(n, steps):
    import numpy as np
    import torch
    from footsies_gym_amd import _abi
    from footsies_gym_amd._lib import check, lib
    from footsies_gym_amd.simulator import FootsiesSim
    from footsies_gym_amd.vector_env import FootsiesEnv, FootsiesVectorEnv
    L = lib()

    def marker():
        torch.cuda.synchronize()
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()

    sim = FootsiesSim(n, p2_mode="external", seed=0)
    h = sim.handle
    p1, p2 = sim.hash_actions(steps + 200, seed=0x5EED)
    torch.cuda.synchronize()
    b1, b2 = p1.data_ptr(), p2.data_ptr()

    def step(k):
        check(L.fs_step(h, C.c_void_p(b1 + k * n), C.c_void_p(b2 + k * n), _abi.FS_ACT_DEVICE), h)

    # "step": bench.py's step_mode / run_step (device rows, back to back, after a warm-up)
    for k in range(200):
        step(k)
    marker()
    for k in range(steps):
        step(200 + k)
    # "step_warm_first": the bench's regions start after a synchronize: the first launches of a
    # region, 20-step regions as the driver's --steps 20 runs them
    marker()
    for r in range(25):
        torch.cuda.synchronize()
        for k in range(20):
            step(k)
    torch.cuda.synchronize()
    # "host_actions": FS_ACT_HOST (pinned staging + H2D copy per step)
    h1, h2 = p1[:500].cpu().numpy(), p2[:500].cpu().numpy()
    marker()
    for k in range(500):
        check(L.fs_step(h, h1[k].ctypes.data, h2[k].ctypes.data, _abi.FS_ACT_HOST), h)
    # "step_gather": fs_step + fs_pack_outputs (the per-step exchange's packing; no collective at 1 GPU)
    rec = torch.empty((n, _abi.FS_RECORD_BYTES), dtype=torch.uint8, device=sim.device)
    marker()
    for k in range(500):
        step(k)
        check(L.fs_pack_outputs(h, C.c_void_p(rec.data_ptr())), h)
    # "step_rec": fs_step_rec (the same records from k_step itself: one launch per step)
    marker()
    recp = C.c_void_p(rec.data_ptr())
    for k in range(500):
        check(L.fs_step_rec(h, C.c_void_p(b1 + k * n), C.c_void_p(b2 + k * n), _abi.FS_ACT_DEVICE, recp), h)
    torch.cuda.synchronize()
    sim.close()
    # the VectorEnv legs (bench.py vector_env_rate): torch output, then numpy output (its kernels
    # write the outputs into pinned host memory)
    rng = np.random.default_rng(0)
    a1 = rng.integers(0, 8, (600, n)).astype(np.uint8)
    a2 = rng.integers(0, 8, (600, n)).astype(np.uint8)
    for kind in ("torch", "numpy"):
        k = [0]
        if kind == "numpy":
            acts, r2 = list(a1), list(a2)
        else:
            acts = list(torch.as_tensor(a1, device="cuda").unbind(0))
            r2 = list(torch.as_tensor(a2, device="cuda").unbind(0))
        env = FootsiesVectorEnv(n, opponent=lambda o, i: r2[k[0]], output=kind, seed=0,
                                retain_host_heap=kind == "numpy")
        env.reset(seed=0)
        marker()
        for j in range(400):
            k[0] = j
            env.step(acts[j])
        marker()
        for j in range(400, 600):
            k[0] = j
            env.step(acts[j])
        torch.cuda.synchronize()
        env.close()
    # "venv_torch_policy": the torch VectorEnv with each step's actions produced on the device just
    # before the step, as a policy's sampling would (the rows are then fresh in L2, not read from HBM)
    g = torch.Generator(device="cuda").manual_seed(0)
    opp = [None]
    env = FootsiesVectorEnv(n, opponent=lambda o, i: opp[0], output="torch", seed=0)
    env.reset(seed=0)
    for leg_steps in (400, 200):  # the warm-up section, then the reported one
        marker()
        for j in range(leg_steps):
            a = torch.randint(0, 8, (n,), generator=g, device="cuda", dtype=torch.uint8)
            opp[0] = torch.randint(0, 8, (n,), generator=g, device="cuda", dtype=torch.uint8)
            env.step(a)
    torch.cuda.synchronize()
    env.close()
    # "single_env": the one-arena FootsiesEnv vs the bot
    env = FootsiesEnv(seed=0)
    env.reset(seed=0)
    acts = [tuple(bool(b) for b in row) for row in rng.integers(0, 2, (520, 3))]
    marker()
    for j in range(20):
        if env.step(acts[j])[2]:
            env.reset()
    marker()
    for j in range(20, 520):
        if env.step(acts[j])[2]:
            env.reset()
    env.close()
    marker()


def reduce(d, out_json):
    import csv
    path = None
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("kernel_trace.csv"):
                path = os.path.join(root, f)
    assert path, "no kernel_trace.csv under %s" % d
    rows = list(csv.DictReader(open(path)))
    key = lambda r: int(r["Start_Timestamp"])  # noqa: E731
    rows.sort(key=key)
    legs, cur = {}, None
    idx = -1
    for r in rows:
        name = r["Kernel_Name"]
        if "spin_kernel" in name:
            idx += 1
            cur = LEGS[idx] if idx < len(LEGS) else None
            continue
        if cur is None or "k_step<" not in name:
            continue
        legs.setdefault(cur, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    out = {"source": os.path.relpath(path, ROOT) if path.startswith(ROOT) else path,
           "command": "rocprofv3 --kernel-trace --output-format csv -- python3 tools/kstep_legs.py", "legs": {}}
    for leg, ds in legs.items():
        if leg.startswith("warm_"):
            continue
        dur = sorted(e - s for s, e, _ in ds)
        starts = [s for s, _, _ in ds]
        gaps = sorted(b - a for a, b in zip(starts, starts[1:]))
        q = lambda v, f: v[min(len(v) - 1, int(f * len(v)))] / 1e3  # noqa: E731
        out["legs"][leg] = {"kernel": ds[0][2], "dispatches": len(ds), "avg_us": sum(dur) / len(dur) / 1e3,
                            "median_us": q(dur, 0.5), "min_us": dur[0] / 1e3, "p99_us": q(dur, 0.99),
                            "max_us": dur[-1] / 1e3,
                            "period_median_us": q(gaps, 0.5) if gaps else None}
    alld = [e - s for leg, ds in legs.items() if not leg.startswith("warm_") for s, e, _ in ds]
    out["all_legs_avg_us"] = sum(alld) / len(alld) / 1e3 if alld else None
    with open(out_json, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--reduce", default=None, help="rocprofv3 output directory to reduce")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    if a.reduce:
        reduce(a.reduce, a.json or os.path.join(ROOT, "profiles", "kstep_legs.json"))
    else:
        run(a.envs, a.steps)


if __name__ == "__main__":
    main()
