"""N>1 path on CPU with gloo (world size 2): contiguous sharding by global arena index with
global-index seeding reproduces the single-process run arena for arena, and the one per-step
collective (the packed all_gather of obs/reward/done) reassembles the global batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from footsies_gym_amd import _abi
from footsies_gym_amd.parallel import gather_outputs, gather_records_to, pack_outputs, shard_range

GLOBAL_N, STEPS = 37, 120


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def actions(t):
    rng = np.random.default_rng(1000 + t)
    return rng.integers(0, 8, GLOBAL_N).astype(np.uint8)


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import binding
    a, b = shard_range(GLOBAL_N, world, rank)
    sizes = [y - x for x, y in (shard_range(GLOBAL_N, world, r) for r in range(world))]
    o = binding.Oracle(b - a, p2_mode=_abi.FS_P2_BOT, base_seed=a)  # seed = global arena index
    gathered, to_root = [], []
    for t in range(STEPS):
        out = o.step(actions(t)[a:b])
        tout = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in out.items() if not k.startswith("final_")}
        g = gather_outputs(tout, shard_sizes=sizes)
        gathered.append({k: v.numpy().copy() for k, v in g.items()})
        r = gather_records_to(pack_outputs(tout, torch), 0, shard_sizes=sizes)  # the learner-only gather
        assert (r is None) == (rank != 0)
        if r is not None:
            to_root.append(r.numpy().copy())
    if rank == 0:
        q.put((gathered, to_root))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_partitions():
    for n, w in [(37, 2), (64, 8), (5, 8), (65536, 8)]:
        rs = [shard_range(n, w, r) for r in range(w)]
        assert rs[0][0] == 0 and rs[-1][1] == n
        assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
        assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


def test_two_rank_gloo_matches_single_process(oracle_lib):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, to_root = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = oracle_lib.Oracle(GLOBAL_N, p2_mode=_abi.FS_P2_BOT, base_seed=0)
    for t in range(STEPS):
        out = ref.step(actions(t))
        for k, v in gathered[t].items():
            assert np.array_equal(np.asarray(out[k]).reshape(v.shape).view(np.uint8), v.view(np.uint8)), (k, t)
        want = pack_outputs({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in out.items()}, torch).numpy()
        assert np.array_equal(to_root[t], want), t


@pytest.mark.parametrize("world", [2, 3, 8])
def test_hashed_shards_are_g_invariant(oracle_lib, world):
    """Shards with arena_base = their first global index draw the global hashed action stream and
    the global creation seeds: G shards == one run, arena for arena (fs_config.arena_base)."""
    n, steps = 50, 150
    ref = oracle_lib.Oracle(n, p2_mode=_abi.FS_P2_BOT, base_seed=7)
    ref.step_n_hashed(steps, 0xD15C)
    want = ref.state()
    got = []
    for r in range(world):
        a, b = shard_range(n, world, r)
        o = oracle_lib.Oracle(b - a, p2_mode=_abi.FS_P2_BOT, base_seed=7, arena_base=a)
        o.step_n_hashed(steps, 0xD15C)
        got.append(o.state())
    assert np.concatenate(got).tobytes() == want.tobytes()


def dp_worker(rank, world, port, q):
    """Data-parallel PPO's host logic over gloo on CPU (no simulator): global advantage statistics,
    the gradient average and PPOTrainer's start (rank 0's weights, equal arena counts)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from footsies_gym_amd.parallel import allreduce_mean_, global_mean_std
    from footsies_gym_amd.ppo import PPOTrainer, make_critic
    from footsies_gym_amd.rollout import make_actor
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(1000 + 337 * rank, generator=g) * (1 + rank) + rank  # uneven shards
    st = global_mean_std(x)
    t = torch.randn(4801, generator=g)
    mine = t.clone()
    allreduce_mean_(t)
    # PPOTrainer's data-parallel start and gradient average (the torch learner's path), without a sim
    tr = PPOTrainer.__new__(PPOTrainer)
    tr.group, tr.world, tr._grad = None, world, None
    tr.actor, tr.critic = make_actor(seed=10 + rank), make_critic(seed=20 + rank)
    tr._join_ranks(64)
    w = torch.cat([p.detach().reshape(-1) for p in list(tr.actor.parameters()) + list(tr.critic.parameters())])
    grads = []
    for p in list(tr.actor.parameters()) + list(tr.critic.parameters()):
        p.grad = torch.randn(p.shape, generator=g)
        grads.append(p.grad.clone().reshape(-1))
    tr._average_grads()
    avg = torch.cat([p.grad.reshape(-1) for p in list(tr.actor.parameters()) + list(tr.critic.parameters())])
    try:
        tr._join_ranks(64 + rank)  # unequal arena counts are refused on every rank
        refused = False
    except ValueError:
        refused = True
    res = {"x": x, "st": st, "t_in": mine, "t": t, "w": w, "g_in": torch.cat(grads), "g": avg}
    res = {k: v.detach().numpy().copy() for k, v in res.items()}  # (arrays, not shared tensors, cross the queue)
    q.put(dict(res, rank=rank, refused=refused))
    dist.barrier()
    dist.destroy_process_group()


def test_data_parallel_ppo_host_logic():
    """ppo.PPOTrainer(group=...)'s collectives on two gloo ranks: the advantage statistics over
    both ranks' (uneven) shards equal torch's mean / std of the concatenation, the gradient
    average is the mean of the ranks' gradients with the same bits on both, the ranks start from
    rank 0's weights, and different arena counts are refused."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(2):
        r = q.get(timeout=120)
        got[r["rank"]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = {r: {k: torch.from_numpy(v) if isinstance(v, np.ndarray) else v for k, v in d.items()} for r, d in got.items()}
    allx = torch.cat([got[0]["x"], got[1]["x"]])
    want = torch.stack([allx.double().mean(), allx.double().std()]).float()
    for r in (0, 1):
        assert torch.allclose(got[r]["st"], want, rtol=1e-6, atol=0), (got[r]["st"], want)
        assert torch.allclose(got[r]["t"], (got[0]["t_in"] + got[1]["t_in"]) / 2, rtol=1e-6, atol=1e-7)
        assert torch.allclose(got[r]["g"], (got[0]["g_in"] + got[1]["g_in"]) / 2, rtol=1e-6, atol=1e-7)
        assert got[r]["refused"]
    assert got[0]["t"].numpy().tobytes() == got[1]["t"].numpy().tobytes()
    assert got[0]["g"].numpy().tobytes() == got[1]["g"].numpy().tobytes()
    assert got[0]["w"].numpy().tobytes() == got[1]["w"].numpy().tobytes()
    from footsies_gym_amd.rollout import make_actor
    from footsies_gym_amd.ppo import make_critic
    w0 = torch.cat([p.detach().reshape(-1) for n in (make_actor(seed=10), make_critic(seed=20)) for p in n.parameters()])
    assert got[1]["w"].numpy().tobytes() == w0.numpy().tobytes()  # rank 0's initial weights
