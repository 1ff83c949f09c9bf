"""Multi-GPU: one process per GPU, arenas sharded by contiguous global index.

Arenas are independent, so stepping needs no communication:
rank r owns global arenas [r*N/G, (r+1)*N/G) and seeds its bots with the global
index, so any G produces the same per-arena trajectories.  The only collective is
the optional per-step gather of (obs, reward, done) for a centralised learner --
one all_gather over RCCL/xGMI of a packed per-arena record (~30 B/arena).
"""
import numpy as np

# packed per-arena record for the gather: guard[2] u8, move[2] u8, action[2] u8, hitstun[2] u8,
# terminated u8, truncated u8, pad[2], move_frame[2] f32, position[2] f32, frame i32, reward f64
RECORD_BYTES = 40


def shard_range(global_envs, world, rank):
    """Contiguous [start, stop) of the global arena index range owned by `rank`."""
    if not 0 <= rank < world:
        raise ValueError("rank %d out of range for world %d" % (rank, world))
    base, extra = divmod(global_envs, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def pack_outputs(out, torch):
    """Outputs dict (torch tensors, [n] / [n,2]) -> one [n, RECORD_BYTES] uint8 tensor."""
    n = out["reward"].shape[0]
    dev = out["reward"].device
    rec = torch.zeros((n, RECORD_BYTES), dtype=torch.uint8, device=dev)
    rec[:, 0:2] = out["guard"]
    rec[:, 2:4] = out["move"]
    rec[:, 4:6] = out["action"]
    rec[:, 6:8] = out["hitstun"]
    rec[:, 8] = out["terminated"]
    rec[:, 9] = out["truncated"]
    rec[:, 12:20] = out["move_frame"].contiguous().view(torch.uint8).view(n, 8)
    rec[:, 20:28] = out["position"].contiguous().view(torch.uint8).view(n, 8)
    rec[:, 28:32] = out["frame"].contiguous().view(torch.uint8).view(n, 4)
    rec[:, 32:40] = out["reward"].contiguous().view(torch.uint8).view(n, 8)
    return rec


def unpack_outputs(rec, torch):
    n = rec.shape[0]
    r = rec.contiguous()
    return {
        "guard": r[:, 0:2].clone(), "move": r[:, 2:4].clone(), "action": r[:, 4:6].clone(),
        "hitstun": r[:, 6:8].clone(), "terminated": r[:, 8].clone(), "truncated": r[:, 9].clone(),
        "move_frame": r[:, 12:20].clone().view(torch.float32).view(n, 2),
        "position": r[:, 20:28].clone().view(torch.float32).view(n, 2),
        "frame": r[:, 28:32].clone().view(torch.int32).view(n),
        "reward": r[:, 32:40].clone().view(torch.float64).view(n),
    }


def gather_records(rec, group=None, shard_sizes=None):
    """All-gather every rank's packed [n, RECORD_BYTES] records into global-index order (one
    all_gather over RCCL/xGMI, or gloo on CPU).  `shard_sizes` (per rank) handles uneven shards
    by padding to the largest.  Returns the [global_envs, RECORD_BYTES] records."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = rec.shape[0]
    sizes = shard_sizes or [n] * world
    m = max(sizes)
    if n < m:
        rec = torch.cat([rec, torch.zeros((m - n, RECORD_BYTES), dtype=rec.dtype, device=rec.device)])
    buf = torch.empty((world * m, RECORD_BYTES), dtype=rec.dtype, device=rec.device)
    dist.all_gather_into_tensor(buf, rec, group=group)
    if all(sz == m for sz in sizes):
        return buf
    return torch.cat([buf[r * m: r * m + sizes[r]] for r in range(world)])


def gather_outputs(out, group=None, shard_sizes=None):
    """All-gather every rank's per-arena outputs dict (torch tensors, any device) into
    global-index order: packed by `pack_outputs`, then `gather_records`."""
    import torch
    return unpack_outputs(gather_records(pack_outputs(out, torch), group, shard_sizes), torch)


class ShardedSim:
    """This rank's FootsiesSim over its shard of `global_envs` arenas (global-index seeding)."""

    def __init__(self, global_envs, rank, world, device=0, seed=0, **kw):
        from .simulator import FootsiesSim
        self.start, self.stop = shard_range(global_envs, world, rank)
        self.sizes = [b - a for a, b in (shard_range(global_envs, world, r) for r in range(world))]
        self.sim = FootsiesSim(self.stop - self.start, device=device, seed=seed + self.start, **kw)

    def step(self, p1, p2=None):
        return self.sim.step(p1, p2)

    def gather(self, group=None):
        """Every rank's outputs in global-index order: the records packed on device by
        fs_pack_outputs, then one all_gather."""
        import torch
        return unpack_outputs(gather_records(self.sim.pack_outputs(), group, self.sizes), torch)

    def close(self):
        self.sim.close()


def global_seeds(global_envs, base_seed=0):
    return np.uint64(base_seed) + np.arange(global_envs, dtype=np.uint64)
