"""Time one C5 minibatch gradient (65 536 arenas x 128 ticks / 4 minibatches = 2 097 152 rows):
fs_ppo_grad (PPOGrad) in both precisions against the same loss through torch autograd (ppo.py
learner="torch", with its SkinnyLinear weight gradients), and fs_ppo_eval in both precisions.  Prints one JSON line."""
import json
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from footsies_gym_amd.ppo import PPOGrad, make_critic, mlp  # noqa: E402
from footsies_gym_amd.rollout import make_actor  # noqa: E402


def main(n=2_097_152, reps=10, only=None):
    dev = torch.device("cuda", 0)
    actor, critic = make_actor(device=dev, seed=1), make_critic(device=dev, seed=2)
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.rand((n, 8), generator=g, device=dev)
    a = torch.randint(0, 8, (n,), generator=g, device=dev).float()
    rows = torch.cat([x, a[:, None], torch.randn((n, 3), generator=g, device=dev) * 0.3], 1).contiguous()
    pg = PPOGrad(actor, critic)
    ps = PPOGrad(actor, critic, precision="split_bf16")
    xe = torch.rand((n + 65536, 8), generator=g, device=dev)
    ae = torch.randint(0, 8, (n + 65536,), generator=g, device=dev).to(torch.uint8)

    def hip():
        pg(rows, 0.2, 0.5, 0.01)

    def hip_split():
        ps(rows, 0.2, 0.5, 0.01)

    def eval_fp32():  # one update's forward passes: values of T + 1 ticks, log-probs of the first
        pg.evaluate(xe, ae, n // 16)

    def eval_split():
        ps.evaluate(xe, ae, n // 16)

    def ref():
        xb, ab = rows[:, :8], rows[:, 8].long()
        lp_all = torch.log_softmax(mlp(actor, xb), dim=1)
        lp = lp_all.gather(1, ab[:, None])[:, 0]
        ratio = torch.exp(lp - rows[:, 9])
        s1, s2 = ratio * rows[:, 10], torch.clamp(ratio, 0.8, 1.2) * rows[:, 10]
        loss = (-torch.min(s1, s2).mean() + 0.5 * (mlp(critic, xb).squeeze(-1) - rows[:, 11]).pow(2).mean()
                - 0.01 * (-(lp_all.exp() * lp_all).sum(1).mean()))
        loss.backward()

    out = {"rows": n}
    for name, fn in (("hip_ms", hip), ("hip_split_ms", hip_split), ("eval_fp32_ms", eval_fp32),
                     ("eval_split_ms", eval_split), ("torch_ms", ref)):
        if only and not name.startswith(only):
            continue
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        out[name] = (time.perf_counter() - t0) / reps * 1e3
    # 2 x (forward 5 120 + backward 4 608 + weight gradients 5 120) fp32 FMAs per row, roughly
    if "hip_ms" in out:
        out["hip_tflops"] = 2 * n * 2 * (5120 + 4608 + 5120) / (out["hip_ms"] * 1e-3) / 1e12
    if "hip_split_ms" in out and "hip_ms" in out:
        out["hip_split_speedup"] = out["hip_ms"] / out["hip_split_ms"]
    if "eval_split_ms" in out and "eval_fp32_ms" in out:
        out["eval_split_speedup"] = out["eval_fp32_ms"] / out["eval_split_ms"]
    print(json.dumps(out))


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=["hip", "torch"])
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    main(reps=a.reps, only=a.only)
