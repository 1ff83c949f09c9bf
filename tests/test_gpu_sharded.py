"""The sharded product path on the GPU: two ranks (processes) sharing cuda:0 over a gloo group,
each a ShardedSim (FootsiesSim with arena_base = its first global index), driven by the fused
hashed-action kernel, per-step device actions and the in-kernel actor, their outputs packed on
device (fs_pack_outputs) and gathered to every rank (all_gather) and to rank 0 (grouped send /
recv) -- all bit-exact against one unsharded FootsiesSim over the global arena count.  (The
driver's 8-GPU runs use the same code over RCCL, one GPU per rank.)"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GLOBAL_N, WORLD, HASHED, STEPS, POLICY = 1000, 2, 120, 25, 40


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def step_actions(t):
    rng = np.random.default_rng(500 + t)
    return rng.integers(0, 8, GLOBAL_N).astype(np.uint8), rng.integers(0, 8, GLOBAL_N).astype(np.uint8)


def run(sim, gather):
    """The scripted sequence on one simulator (a ShardedSim shard or the global FootsiesSim);
    `gather()` returns the global outputs dict (numpy) or None."""
    import torch
    from footsies_gym_amd.rollout import FusedPolicyRollout, make_actor
    base, stop = getattr(sim, "start", 0), getattr(sim, "stop", GLOBAL_N)
    inner = getattr(sim, "sim", sim)
    res = {"gathered": []}
    inner.step_n(HASHED, None, None, action_seed=0x5AD)   # fused, in-kernel hashed actions
    for t in range(STEPS):                                 # per-step device actions
        a1, a2 = step_actions(t)
        inner.step(torch.as_tensor(a1[base:stop], device=inner.device),
                   torch.as_tensor(a2[base:stop], device=inner.device))
        res["gathered"].append(gather())
    _, q2 = inner.hash_actions(POLICY, seed=0xB0B)         # P2's rows, keyed by global index too
    ro = FusedPolicyRollout(inner, make_actor(device=inner.device, seed=3), seed=8)
    acts, logp = ro.rollout(POLICY, p2_actions=q2)        # the in-kernel actor's sampling stream
    torch.cuda.synchronize()
    res["policy_actions"] = acts.cpu().numpy()
    res["state"] = inner.get_state()
    return res


def worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from footsies_gym_amd.parallel import ShardedSim
    sim = ShardedSim(GLOBAL_N, rank, WORLD, device=0, seed=3, p2_mode="external")

    def gather():
        every = {k: v.cpu().numpy() for k, v in sim.gather().items()}
        root = sim.gather(dst=0)
        if root is not None:
            root = {k: v.cpu().numpy() for k, v in root.items()}
        return every, root
    res = run(sim, gather)
    res["rank"] = rank
    q.put(res)
    dist.barrier()
    sim.close()
    dist.destroy_process_group()


BENCH_N, BENCH_LAUNCHES = 4096, [5] + [20] * 5 + [7]


def bench_flow(n, arena_base):
    """What bench.py does on each rank: FootsiesSim(arena_base = rank * N), the hashed rows of
    its own global arenas written to HBM (fs_hash_actions), then consecutive fs_step_n_packed
    launches into one reused packed trajectory.  Returns every launch's records and the state."""
    import torch
    from footsies_gym_amd.simulator import FootsiesSim
    sim = FootsiesSim(n, device=0, p2_mode="external", seed=0, arena_base=arena_base)
    total = sum(BENCH_LAUNCHES)
    p1, p2 = sim.hash_actions(total, seed=0x5EED, t0=0)
    traj = sim.alloc_packed_trajectory(max(BENCH_LAUNCHES))
    recs, k = [], 0
    for m in BENCH_LAUNCHES:
        sim.step_n_packed(m, p1[k:k + m], p2[k:k + m], trajectory=traj)
        torch.cuda.synchronize()
        recs.append({key: v[:m].cpu().numpy() for key, v in traj.items()})
        k += m
    state = sim.get_state()
    sim.close()
    return recs, state


def bench_worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    recs, state = bench_flow(BENCH_N, rank * BENCH_N)
    q.put({"rank": rank, "recs": recs, "state": state})
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_bench_flow_match_unsharded():
    """bench.py's per-rank flow (hashed rows keyed by global index, packed fused launches of the
    driver's shape) on two ranks sharing cuda:0: the ranks' records and states, concatenated in
    rank order, equal one unsharded 2N-arena handle's byte for byte."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=bench_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(WORLD):
        r = q.get(timeout=240)
        got[r["rank"]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    recs, state = bench_flow(WORLD * BENCH_N, 0)
    assert np.concatenate([got[r]["state"] for r in range(WORLD)]).tobytes() == state.tobytes()
    for j, want in enumerate(recs):
        for key, v in want.items():
            shard = np.concatenate([got[r]["recs"][j][key] for r in range(WORLD)], axis=1)
            assert shard.tobytes() == v.tobytes(), (j, key)
    assert any(w["lanes"][..., 1, 12].any() for w in recs)  # rounds ended (final records written)


def test_two_ranks_on_one_gpu_match_unsharded():
    import torch.multiprocessing as mp
    from footsies_gym_amd.parallel import unpack_outputs
    from footsies_gym_amd.simulator import FootsiesSim
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(WORLD):
        r = q.get(timeout=240)
        got[r["rank"]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import torch
    ref_sim = FootsiesSim(GLOBAL_N, device=0, seed=3, p2_mode="external")
    ref = run(ref_sim, lambda: {k: v.cpu().numpy() for k, v in
                                unpack_outputs(ref_sim.pack_outputs(), torch).items()})
    assert np.concatenate([got[r]["state"] for r in range(WORLD)]).tobytes() == ref["state"].tobytes()
    assert np.array_equal(np.concatenate([got[r]["policy_actions"] for r in range(WORLD)], axis=1),
                          ref["policy_actions"])
    for t in range(STEPS):
        want = ref["gathered"][t]
        for r in range(WORLD):
            every, root = got[r]["gathered"][t]
            assert (root is not None) == (r == 0)
            for k, v in want.items():
                assert every[k].tobytes() == v.tobytes(), (t, r, k)
                if root is not None:
                    assert root[k].tobytes() == v.tobytes(), (t, k)
    ref_sim.close()
