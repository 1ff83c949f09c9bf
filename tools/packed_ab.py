#!/usr/bin/env python3
"""fs_step_n into a per-field trajectory vs fs_step_n_packed into a packed one (include/footsies.h
fs_packed_traj), same handle shape, same action rows: the median launch time by HIP events on the
launch stream, interleaved rounds (measurement only, GPU box).

  python tools/packed_ab.py [--envs 65536 32768] [--ticks 1000 20] [--rounds 3] [--p2 external bot]

(From 131 072 arenas both layouts run the one-lane kernels: k_step_n1 / k_step_n1_packed.)
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, nargs="+", default=[65536, 32768])
    ap.add_argument("--ticks", type=int, nargs="+", default=[1000, 20])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--launches", type=int, default=7)
    ap.add_argument("--p2", nargs="+", default=["external"], choices=["external", "bot"])
    a = ap.parse_args()
    import torch
    from footsies_gym_amd.simulator import FootsiesSim
    from footsies_gym_amd import _abi
    from footsies_gym_amd._lib import lib
    for n, T, mode in [(n, T, m) for m in a.p2 for n in a.envs for T in a.ticks]:
        if True:
            sims = {k: FootsiesSim(n, p2_mode=mode, seed=0) for k in ("per_field", "packed")}
            p1, p2 = sims["per_field"].hash_actions(T, seed=0x5EED, p2=mode == "external")
            bufs = {"per_field": sims["per_field"].alloc_trajectory(T), "packed": sims["packed"].alloc_packed_trajectory(T)}
            run = {"per_field": lambda: sims["per_field"].step_n(T, p1, p2, trajectory=bufs["per_field"]),
                   "packed": lambda: sims["packed"].step_n_packed(T, p1, p2, trajectory=bufs["packed"])}
            for f in run.values():
                f()
            torch.cuda.synchronize()
            res = {k: [] for k in run}
            for r in range(a.rounds):
                for k, f in run.items():
                    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                           for _ in range(a.launches)]
                    torch.cuda._sleep(int(2e7))
                    for e0, e1 in evs:
                        e0.record()
                        f()
                        e1.record()
                    torch.cuda.synchronize()
                    d = sorted(e0.elapsed_time(e1) * 1e3 for e0, e1 in evs)
                    res[k].append(d[len(d) // 2])
            med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
            kn = {k: lib().fs_step_kernel(sims[k].handle, T, f).decode()
                  for k, f in (("per_field", 0), ("packed", _abi.FS_KERNEL_PACKED))}
            print("P2=%s N=%d ticks=%d  per-field %.1f us (%.3e env-steps/s, %s)  packed %.1f us (%.3e, %s)  packed %+.1f%%" % (
                mode, n, T, med["per_field"], n * T / med["per_field"] * 1e6, kn["per_field"], med["packed"],
                n * T / med["packed"] * 1e6, kn["packed"], 100 * (med["per_field"] / med["packed"] - 1)), flush=True)
            for s in sims.values():
                s.close()
            del bufs


if __name__ == "__main__":
    main()
