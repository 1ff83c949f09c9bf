#!/usr/bin/env python3
"""Time the torch glue of one PPO iteration at C5's size (measurement only, on a GPU box):
the feature build from a [T][N] trajectory and the [M, 12] sample table, each as torch.cat and
as writes into column views of one preallocated buffer; checks the two agree bit for bit.

  python tools/ppo_glue_time.py [--envs 65536] [--horizon 128]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--horizon", type=int, default=128)
    args = ap.parse_args()
    T, N, dev = args.horizon, args.envs, torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    tr = {"guard": torch.randint(0, 4, (T, N, 2), generator=g, device=dev, dtype=torch.uint8),
          "move": torch.randint(0, 17, (T, N, 2), generator=g, device=dev, dtype=torch.uint8),
          "move_frame": torch.randint(0, 56, (T, N, 2), generator=g, device=dev).float(),
          "position": torch.rand((T, N, 2), generator=g, device=dev) * 9 - 4.5}
    feats_a = torch.empty((T + 1, N, 8), device=dev)
    feats_b = torch.empty((T + 1, N, 8), device=dev)

    def f_cat():
        feats_a[1:] = torch.cat([tr["guard"].float() / 3.0, tr["move"].float() / 16.0, tr["move_frame"] / 55.0,
                                 tr["position"] / 4.6], dim=2)

    def f_views():
        f = feats_b[1:]
        torch.div(tr["guard"], 3.0, out=f[..., 0:2])
        torch.div(tr["move"], 16.0, out=f[..., 2:4])
        torch.div(tr["move_frame"], 55.0, out=f[..., 4:6])
        torch.div(tr["position"], 4.6, out=f[..., 6:8])

    t_cat, t_views = timeit(f_cat), timeit(f_views)
    same_f = torch.equal(feats_a[1:], feats_b[1:])

    M = T * N
    x = feats_a[:T].reshape(M, 8)
    a = torch.randint(0, 8, (M,), generator=g, device=dev)
    old, adv, ret = (torch.randn(M, generator=g, device=dev) for _ in range(3))
    rows_b = torch.empty((M, 12), device=dev)
    holder = {}

    def r_cat():
        holder["a"] = torch.cat([x, a[:, None].float(), old[:, None], adv[:, None], ret[:, None]], dim=1)

    def r_views():
        rows_b[:, :8].copy_(x)
        rows_b[:, 8].copy_(a)
        rows_b[:, 9].copy_(old)
        rows_b[:, 10].copy_(adv)
        rows_b[:, 11].copy_(ret)

    t_rcat, t_rviews = timeit(r_cat), timeit(r_views)
    same_r = torch.equal(holder["a"], rows_b)
    from footsies_gym_amd.ppo import gae
    rew, don = torch.randn((T, N), generator=g, device=dev), (torch.rand((T, N), generator=g, device=dev) < 0.01).float()
    val = torch.randn((T + 1, N), generator=g, device=dev)
    t_gae = timeit(lambda: gae(rew, val, don, 0.99, 0.95))
    print({"gae_ms": round(t_gae, 4), "features_cat_ms": round(t_cat, 4), "features_views_ms": round(t_views, 4), "features_equal": same_f,
           "rows_cat_ms": round(t_rcat, 4), "rows_views_ms": round(t_rviews, 4), "rows_equal": same_r})


if __name__ == "__main__":
    main()
