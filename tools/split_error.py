#!/usr/bin/env python3
"""Accuracy of fs_ppo_grad's two precisions (measurement only): per gradient tensor, the largest
|kernel - reference| / max|reference| and the largest elementwise relative error over the
elements above 1e-3 x max|reference|, the reference being the same loss through autograd in
float64.  torch fp32 autograd is listed beside them.  Prints one JSON line per sample count,
with rows as drawn and with rows kept 1e-3 away from the clip edges (tests/test_gpu_learn._rows)."""
import copy
import json
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_learn import _nets, _rows, _torch_reference  # noqa: E402
from footsies_gym_amd.ppo import PPOGrad  # noqa: E402

NAMES = ["actor.w1", "actor.b1", "actor.w2", "actor.b2", "actor.w3", "actor.b3",
         "critic.w1", "critic.b1", "critic.w2", "critic.b2", "critic.w3", "critic.b3"]


def errs(got, ref):
    out = {}
    for name, g, e in zip(NAMES, got, ref):
        g, e = g.double(), e.double()
        scale = float(e.abs().max())
        d = (g - e).abs()
        big = e.abs() > 1e-3 * scale
        out[name] = [float(d.max()) / scale, float((d[big] / e.abs()[big]).max()) if bool(big.any()) else 0.0]
    return out


for n, margin in ((5000, 0.0), (70001, 0.0), (1_000_000, 0.0), (70001, 1e-3), (1_000_000, 1e-3)):
    actor, critic = _nets(seed=n % 7)
    rows = _rows(actor, n, seed=n, margin=margin)
    a64, c64 = copy.deepcopy(actor).double(), copy.deepcopy(critic).double()
    ref, _ = _torch_reference(a64, c64, rows.double(), 0.2, 0.5, 0.01)
    t32, _ = _torch_reference(actor, critic, rows, 0.2, 0.5, 0.01)
    res = {"n": n, "clip_edge_margin": margin, "torch_fp32": errs(t32, ref)}
    for prec in ("fp32", "split_bf16"):
        pg = PPOGrad(actor, critic, precision=prec)
        pg(rows, 0.2, 0.5, 0.01)
        res[prec] = errs([p.grad.detach().clone() for p in pg.params], ref)
    torch.cuda.synchronize()
    print(json.dumps(res))
