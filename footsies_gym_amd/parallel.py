"""Multi-GPU: one process per GPU, arenas sharded by contiguous global index.

Arenas are independent, so stepping needs no communication:
rank r owns global arenas [r*N/G, (r+1)*N/G); its handle's arena_base is r*N/G, so
seeds, hashed actions and actor samples are keyed by the global index and any G
produces the same per-arena trajectories.  The only collective is the optional
per-step gather of (obs, reward, done) for a centralised learner: a packed 40-B
per-arena record, all-gathered to every rank or gathered to one rank by grouped
point-to-point sends over RCCL/xGMI.  Data-parallel PPO (ppo.PPOTrainer(group=...)) keeps its
rollouts rank-local and averages each minibatch's gradient (`allreduce_mean_`) and the advantage
statistics (`global_mean_std`) over the ranks.
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


def _on_backend(t, group):
    """gloo moves host tensors only: records of a device shard cross through host memory there
    (the multi-rank rehearsal on one GPU); RCCL takes them where they are."""
    import torch.distributed as dist
    return t.cpu() if t.is_cuda and dist.get_backend(group) == "gloo" else t


def gather_records(rec, group=None, shard_sizes=None):
    """All-gather every rank's packed [n, RECORD_BYTES] records into global-index order (one
    all_gather over RCCL/xGMI, or gloo on CPU).  `shard_sizes` (per rank) handles uneven shards
    by padding to the largest.  Returns the [global_envs, RECORD_BYTES] records on every rank."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = rec.shape[0]
    sizes = shard_sizes or [n] * world
    m = max(sizes)
    dev = rec.device
    rec = _on_backend(rec, group)
    if n < m:
        rec = torch.cat([rec, torch.zeros((m - n, RECORD_BYTES), dtype=rec.dtype, device=rec.device)])
    buf = torch.empty((world * m, RECORD_BYTES), dtype=rec.dtype, device=rec.device)
    dist.all_gather_into_tensor(buf, rec, group=group)
    if not all(sz == m for sz in sizes):
        buf = torch.cat([buf[r * m: r * m + sizes[r]] for r in range(world)])
    return buf.to(dev)


def gather_records_to(rec, dst=0, group=None, shard_sizes=None):
    """Gather every rank's packed records to rank `dst` only (a centralised learner, SURVEY.md
    §8(e)): one grouped point-to-point exchange -- each rank sends its shard, `dst` posts one
    receive per peer straight into its slice of the global buffer (RCCL has no native gather; this
    is the ncclGroupStart + ncclSend / ncclRecv pattern).  Each link carries one shard once, so
    the traffic is (G-1)/G of what `gather_records`'s all_gather moves into every rank.  Returns
    the [global_envs, RECORD_BYTES] records on `dst`, None elsewhere."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = rec.shape[0]
    sizes = shard_sizes or [n] * world
    starts = np.concatenate([[0], np.cumsum(sizes)]).astype(int)
    dev = rec.device
    rec = _on_backend(rec.contiguous(), group)
    if rank != dst:  # (a batch on every rank: with RCCL, the first P2P batch of a group must include all ranks)
        for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, rec, dst, group=group)]):
            w.wait()
        return None
    out = torch.empty((int(starts[-1]), RECORD_BYTES), dtype=rec.dtype, device=rec.device)
    out[starts[rank]:starts[rank + 1]] = rec
    ops = [dist.P2POp(dist.irecv, out[starts[r]:starts[r + 1]], r, group=group) for r in range(world) if r != dst]
    for w in dist.batch_isend_irecv(ops) if ops else []:
        w.wait()
    return out.to(dev)


def gather_outputs(out, group=None, shard_sizes=None):
    """All-gather every rank's per-arena outputs dict (torch tensors, any device) into
    global-index order: packed by `pack_outputs`, then `gather_records`."""
    import torch
    return unpack_outputs(gather_records(pack_outputs(out, torch), group, shard_sizes), torch)


class ShardedSim:
    """This rank's FootsiesSim over its shard of `global_envs` arenas.  The handle's arena_base is
    the shard's first global index, so creation seeds, hashed actions and the in-kernel actor's
    sampling stream are those of the same arenas in one unsharded run: results do not depend on G."""

    def __init__(self, global_envs, rank, world, device=0, seed=0, **kw):
        from .simulator import FootsiesSim
        self.start, self.stop = shard_range(global_envs, world, rank)
        self.sizes = [b - a for a, b in (shard_range(global_envs, world, r) for r in range(world))]
        self.sim = FootsiesSim(self.stop - self.start, device=device, seed=seed, arena_base=self.start, **kw)

    def step(self, p1, p2=None):
        return self.sim.step(p1, p2)

    def step_n(self, n, p1=None, p2=None, action_seed=0, trajectory=None):
        return self.sim.step_n(n, p1, p2, action_seed=action_seed, trajectory=trajectory)

    def gather(self, group=None, dst=None):
        """The outputs of every rank in global-index order, packed on device by fs_pack_outputs:
        on every rank (one all_gather, dst=None) or on rank `dst` only (grouped send / recv;
        None on the other ranks)."""
        import torch
        rec = self.sim.pack_outputs()
        if dst is None:
            return unpack_outputs(gather_records(rec, group, self.sizes), torch)
        g = gather_records_to(rec, dst, group, self.sizes)
        return None if g is None else unpack_outputs(g, torch)

    def step_gather(self, p1, p2=None, group=None, dst=None):
        """step() and gather() in one: the step's kernel writes the records (fs_step_rec) that
        gather() would pack, then the same all_gather (dst=None) or send / recv to rank dst."""
        import torch
        rec = self.sim.step_records(p1, p2)
        if dst is None:
            return unpack_outputs(gather_records(rec, group, self.sizes), torch)
        g = gather_records_to(rec, dst, group, self.sizes)
        return None if g is None else unpack_outputs(g, torch)

    def close(self):
        self.sim.close()


def allreduce_mean_(t, group=None):
    """Data-parallel PPO's one exchange (rollouts stay rank-local, gradients are
    averaged): `t` replaced in place by its mean over the ranks -- one all_reduce SUM over
    RCCL / xGMI (through host memory with gloo), then / world.  Every rank ends with the same bits
    (the collective's result is the same buffer on all of them).  Returns `t`."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if world == 1:
        return t
    x = _on_backend(t, group)
    dist.all_reduce(x, op=dist.ReduceOp.SUM, group=group)
    x.div_(world)
    if x is not t:
        t.copy_(x)
    return t


def global_mean_std(x, group=None):
    """Mean and unbiased standard deviation of the union of every rank's `x` (any shapes; ranks
    may hold different counts), as a float32 [2] tensor on x's device: float64 sums, two
    all_reduces of two scalars -- the global count and sum, then the squared deviations from the
    global mean (the two-pass form torch.std uses on one tensor)."""
    import torch
    import torch.distributed as dist
    xd = x.reshape(-1).double()
    a = _on_backend(torch.stack([torch.tensor(float(xd.numel()), dtype=torch.float64, device=x.device), xd.sum()]),
                    group)
    dist.all_reduce(a, op=dist.ReduceOp.SUM, group=group)
    n, mean = a[0].to(x.device), (a[1] / a[0]).to(x.device)
    m2 = _on_backend(((xd - mean) ** 2).sum().reshape(1), group)
    dist.all_reduce(m2, op=dist.ReduceOp.SUM, group=group)
    std = (m2[0].to(x.device) / (n - 1)).sqrt()
    return torch.stack([mean, std]).float()


def global_seeds(global_envs, base_seed=0):
    return np.uint64(base_seed) + np.arange(global_envs, dtype=np.uint64)
