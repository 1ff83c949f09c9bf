"""Data-parallel PPO on the GPU (rollouts rank-local, gradients averaged): two
ranks sharing cuda:0 over a gloo group, each a PPOTrainer(group=...) over its own 4 096 arenas
(arena_base = rank x 4 096).  The ranks start from rank 0's weights and stay bit-identical through
training; the advantages are normalised over both ranks together; and one minibatch's averaged
gradient equals fs_ppo_grad over both ranks' minibatch rows in one call, up to fp32 summation
order.  (The driver's multi-GPU bench runs the same trainer over RCCL: bench.py's ppo_dp leg.)"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, T, WORLD, K = 4096, 32, 2, 16384


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def flat_weights(tr):
    import torch
    return torch.cat([p.detach().reshape(-1) for p in list(tr.actor.parameters()) + list(tr.critic.parameters())])


def worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from footsies_gym_amd.parallel import allreduce_mean_
    from footsies_gym_amd.ppo import PPOGrad, PPOTrainer
    from footsies_gym_amd.simulator import FootsiesSim
    sim = FootsiesSim(N, device=0, p2_mode="bot", seed=0, arena_base=rank * N)
    # seed = rank: each rank would draw its own initial weights; the trainer starts from rank 0's
    tr = PPOTrainer(sim, horizon=T, group="default", learner_precision="fp32", seed=rank)
    w0 = flat_weights(tr).cpu().numpy()
    tr.train(2)
    w2 = flat_weights(tr).cpu().numpy()
    loss = tr.stats["loss"].item()
    rows, _ = tr.prepare(*tr.collect())
    mb = rows[:K].contiguous()
    pg = PPOGrad(tr.actor, tr.critic, precision="fp32")
    pg(mb, tr.clip, tr.vf_coef, tr.ent_coef)
    g_local = pg.grad.clone()
    g_dp = allreduce_mean_(pg.grad.clone()).cpu().numpy()
    every = [torch.zeros_like(mb.cpu()) for _ in range(WORLD)]
    dist.all_gather(every, mb.cpu())
    pg(torch.cat(every).to(mb.device).contiguous(), tr.clip, tr.vf_coef, tr.ent_coef)
    g_cat = pg.grad.cpu().numpy()
    adv = rows[:, 10].cpu()
    advs = [torch.zeros_like(adv) for _ in range(WORLD)]
    dist.all_gather(advs, adv)
    q.put({"rank": rank, "w0": w0, "w2": w2, "loss": loss, "g_dp": g_dp, "g_cat": g_cat,
           "g_local": g_local.cpu().numpy(), "adv": torch.cat(advs).numpy(), "own_adv_mean": float(adv.mean())})
    sim.close()
    dist.barrier()
    dist.destroy_process_group()


def test_data_parallel_ppo_two_ranks_on_one_gpu():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(WORLD):
        r = q.get(timeout=300)
        got[r["rank"]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    a, b = got[0], got[1]
    # rank 0's initial weights on both ranks; identical updates keep them identical; they moved
    assert a["w0"].tobytes() == b["w0"].tobytes()
    assert a["w2"].tobytes() == b["w2"].tobytes()
    assert not np.array_equal(a["w0"], a["w2"])
    assert a["loss"] == b["loss"]
    # the ranks' minibatches differ (different arenas), their average is the joint minibatch's gradient
    assert not np.array_equal(a["g_local"], b["g_local"])
    assert a["g_dp"].tobytes() == b["g_dp"].tobytes()
    scale = np.abs(a["g_cat"]).max()
    assert np.abs(a["g_dp"] - a["g_cat"]).max() <= 2e-5 * scale, (np.abs(a["g_dp"] - a["g_cat"]).max(), scale)
    # advantages normalised over both ranks together (each rank alone is not centred)
    adv = a["adv"].astype(np.float64)
    assert abs(adv.mean()) < 1e-5 and abs(adv.std(ddof=1) - 1.0) < 1e-4, (adv.mean(), adv.std(ddof=1))
    assert max(abs(a["own_adv_mean"]), abs(b["own_adv_mean"])) > 1e-4
