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
