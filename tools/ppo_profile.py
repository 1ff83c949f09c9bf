#!/usr/bin/env python3
"""Phase timing of one PPO iteration (measurement only, on a GPU box).

  python tools/ppo_profile.py [--envs 65536] [--horizon 128]

Prints the wall time of each phase of footsies_gym_amd.ppo.PPOTrainer (fused rollout, critic
pass, GAE, minibatch update) over two iterations, then a torch.profiler table of one more
iteration, sorted by device time.  DESIGN.md's PPO section quotes these phases.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--horizon", type=int, default=128)
    args = ap.parse_args()
    import torch
    from torch.profiler import ProfilerActivity, profile

    from footsies_gym_amd.ppo import PPOTrainer, gae_device
    from footsies_gym_amd.rollout import N_FEATURES
    from footsies_gym_amd.simulator import FootsiesSim

    sim = FootsiesSim(args.envs, device=0, p2_mode="bot", seed=0)
    tr = PPOTrainer(sim, horizon=args.horizon)
    tr.train(1)  # warm-up

    def now():
        torch.cuda.synchronize()
        return time.perf_counter()

    for _ in range(2):
        a = now()
        feats, actions, rewards, dones = tr.collect()
        b = now()
        with torch.no_grad():  # the trainer's own launches (learner="hip")
            values, _ = tr._grad.evaluate(feats.view(-1, N_FEATURES))
            c = now()
            gae_device(rewards, dones, values.view(-1, sim.num_envs), tr.gamma, tr.lam)
            d = now()
        tr.update(feats, actions, rewards, dones)
        e = now()
        print("collect %.1f ms, critic %.1f ms, gae %.1f ms, update (incl. its own critic + gae) %.1f ms"
              % ((b - a) * 1e3, (c - b) * 1e3, (d - c) * 1e3, (e - d) * 1e3), flush=True)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        tr.iterate()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25))
    sim.close()


if __name__ == "__main__":
    main()
