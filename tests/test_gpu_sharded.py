"""The sharded product path on the GPU: two ranks (processes) sharing cuda:0 over a gloo group,
each a ShardedSim (FootsiesSim with arena_base = its first global index), driven by the fused
hashed-action kernel, per-step device actions and the in-kernel actor, their outputs packed on
device (fs_pack_outputs) and gathered to every rank (all_gather) and to rank 0 (grouped send /
recv) -- all bit-exact against one unsharded FootsiesSim over the global arena count.  (The
driver's 8-GPU runs use the same code over RCCL, one GPU per rank.)"""
import hashlib
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
# bench.py's c4_strong leg at N = 2: 262 144 arenas as 2 x 131 072 (arena_base = rank x 131 072), the
# driver's launch shape (5 warm-up ticks, 20-tick regions) then one LEG_TICKS-tick launch
C4_N, C4_LAUNCHES, C4_TAIL = 131072, [5, 20, 20, 1000], 40


def bench_flow(n, arena_base, launches=BENCH_LAUNCHES, tail=None, shards=1):
    """What bench.py does on each rank: FootsiesSim(arena_base = rank * N), the hashed rows of
    its own global arenas written to HBM (fs_hash_actions), then consecutive fs_step_n_packed
    launches into one reused packed trajectory.  Returns every launch's records (the last `tail`
    ticks of each when given) and the state; with shards > 1 each record array and the state
    are split along the arena axis into that many equal parts (one per rank of a sharded run)."""
    import torch
    from footsies_gym_amd.simulator import FootsiesSim
    sim = FootsiesSim(n, device=0, p2_mode="external", seed=0, arena_base=arena_base)
    total = sum(launches)
    p1, p2 = sim.hash_actions(total, seed=0x5EED, t0=0)
    traj = sim.alloc_packed_trajectory(max(launches))
    recs, k = [], 0
    for m in launches:
        sim.step_n_packed(m, p1[k:k + m], p2[k:k + m], trajectory=traj)
        torch.cuda.synchronize()
        lo = 0 if tail is None else max(0, m - tail)
        recs.append({key: v[lo:m].cpu().numpy() for key, v in traj.items()})
        k += m
    state = sim.get_state()
    sim.close()
    del p1, p2, traj
    torch.cuda.empty_cache()
    if shards > 1:
        recs = [{key: np.split(v, shards, axis=1) for key, v in r.items()} for r in recs]
        state = np.split(state, shards)
    return recs, state


def bench_worker(rank, port, q, n=BENCH_N, launches=BENCH_LAUNCHES, tail=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    recs, state = bench_flow(n, rank * n, launches, tail)
    if tail is not None:  # large shards: digests cross the queue, not the arrays
        recs = [{key: hashlib.sha256(v.tobytes()).hexdigest() for key, v in r.items()} for r in recs]
        state = hashlib.sha256(state.tobytes()).hexdigest()
    q.put({"rank": rank, "recs": recs, "state": state})
    dist.barrier()
    dist.destroy_process_group()


def run_bench_ranks(**kw):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=bench_worker, args=(r, port, q), kwargs=kw) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(WORLD):
        r = q.get(timeout=240)
        got[r["rank"]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


def test_two_ranks_bench_flow_match_unsharded():
    """bench.py's per-rank flow (hashed rows keyed by global index, packed fused launches of the
    driver's shape) on two ranks sharing cuda:0: the ranks' records and states, concatenated in
    rank order, equal one unsharded 2N-arena handle's byte for byte."""
    got = run_bench_ranks()
    recs, state = bench_flow(WORLD * BENCH_N, 0)
    assert np.concatenate([got[r]["state"] for r in range(WORLD)]).tobytes() == state.tobytes()
    for j, want in enumerate(recs):
        for key, v in want.items():
            shard = np.concatenate([got[r]["recs"][j][key] for r in range(WORLD)], axis=1)
            assert shard.tobytes() == v.tobytes(), (j, key)
    assert any(w["lanes"][..., 1, 12].any() for w in recs)  # rounds ended (final records written)


def test_c4_strong_split_matches_unsharded():
    """bench.py's c4_strong leg at N = 2: two ranks of 131 072 arenas each
    (arena_base 0 and 131 072) through the leg's launches -- the driver's 5-tick warm-up and 20-tick
    regions, then a 1000-tick launch -- against one unsharded 262 144-arena handle: each rank's
    half of every launch's records (the last 40 ticks of each) and of the final state, byte for
    byte (SHA-256 of each half)."""
    got = run_bench_ranks(n=C4_N, launches=C4_LAUNCHES, tail=C4_TAIL)
    recs, state = bench_flow(WORLD * C4_N, 0, C4_LAUNCHES, C4_TAIL, shards=WORLD)
    digest = lambda a: hashlib.sha256(a.tobytes()).hexdigest()  # noqa: E731
    for r in range(WORLD):
        assert got[r]["state"] == digest(state[r]), r
        for j, want in enumerate(recs):
            for key, parts in want.items():
                assert got[r]["recs"][j][key] == digest(parts[r]), (r, j, key)
    assert any(w["lanes"][1][..., 1, 12].any() for w in recs)  # rounds ended in the second half too


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
