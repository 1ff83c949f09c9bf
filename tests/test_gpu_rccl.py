"""RCCL (the `nccl` backend) executing on the GPU box: a one-rank process group on cuda:0.

The driver's scaling runs use RCCL with one GPU per rank; this box has one GPU, so these tests
run the same calls at world size 1, where RCCL still runs its own kernels and copies:
* `bench.py --gpus 1` under `torch.distributed.run` (a launcher, so bench joins a process group):
  barrier, the max-over-ranks all_reduce, the per-step all_gather of packed records and the
  grouped send / recv path, with the line reporting backend "nccl" and world size 1;
* `ShardedSim.gather()` (all_gather_into_tensor) and `gather(dst=0)` over RCCL return exactly the
  shard's own packed outputs."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_under_launcher_runs_rccl_at_world_one():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", "--master-port=%d" % free_port(), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "20", "--warmup", "5", "--envs", "4096", "--roofline-ticks", "20",
           "--kernel-samples", "5", "--no-cpu-baseline", "--no-extras"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["ranks"]["world_size"] == 1
    assert line["ranks"]["backend"] == "nccl"
    assert line["value"] > 0 and line["step_gather_mode"]["value"] > 0
    assert line["step_gather_mode"]["bytes_gathered_per_step"] == 4096 * 40


def test_plain_one_gpu_bench_gathers_over_rccl():
    """The driver's plain `bench.py --gpus 1` (no launcher) forms a one-rank RCCL group, so its per-step
    gather leg runs the all_gather; --no-solo-group keeps the old ungrouped run."""
    args = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "20", "--warmup", "5",
            "--envs", "4096", "--roofline-ticks", "20", "--kernel-samples", "5", "--no-cpu-baseline", "--no-extras",
            "--no-c4"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    lines = []
    for extra in ([], ["--no-solo-group"]):
        out = subprocess.run(args + extra, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
        assert out.returncode == 0, out.stderr[-2000:]
        lines.append(json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]))
    solo, plain = lines
    assert solo["ranks"]["backend"] == "nccl" and solo["ranks"]["world_size"] == 1 and not solo["ranks"]["launcher"]
    assert solo["step_gather_mode"]["collective"] is True and solo["ranks"]["solo_group_error"] is None
    assert plain["ranks"]["backend"] is None and plain["step_gather_mode"]["collective"] is False
    assert solo["value"] > 0 and plain["value"] > 0


def _worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from footsies_gym_amd.parallel import ShardedSim, unpack_outputs
    sim = ShardedSim(777, 0, 1, device=0, seed=5, p2_mode="bot")
    sim.sim.step_n(37, None, None, action_seed=0x77)  # hashed P1 actions, P2 = the bot
    every = {k: v.cpu().numpy() for k, v in sim.gather().items()}
    root = {k: v.cpu().numpy() for k, v in sim.gather(dst=0).items()}
    local = {k: v.cpu().numpy() for k, v in unpack_outputs(sim.sim.pack_outputs(), torch).items()}
    # step_gather: the step kernel writes the records (fs_step_rec), then the same collectives
    a1 = torch.full((777,), 3, dtype=torch.uint8, device="cuda:0")
    sg = {k: v.cpu().numpy() for k, v in sim.step_gather(a1).items()}
    sg_local = {k: v.cpu().numpy() for k, v in unpack_outputs(sim.sim.pack_outputs(), torch).items()}
    sg_root = {k: v.cpu().numpy() for k, v in sim.step_gather(a1, dst=0).items()}
    sg_local2 = {k: v.cpu().numpy() for k, v in unpack_outputs(sim.sim.pack_outputs(), torch).items()}
    dist.barrier()
    q.put({"backend": dist.get_backend(), "every": every, "root": root, "local": local,
           "sg": (sg, sg_local), "sg_root": (sg_root, sg_local2)})
    sim.close()
    dist.destroy_process_group()


def test_sharded_gather_over_rccl_world_one():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(free_port(), q))
    p.start()
    r = q.get(timeout=100)
    p.join(timeout=30)
    assert p.exitcode == 0
    assert r["backend"] == "nccl"
    for k, v in r["local"].items():
        assert r["every"][k].tobytes() == v.tobytes(), k
        assert r["root"][k].tobytes() == v.tobytes(), k
    assert np.any(r["local"]["frame"] != 0)
    for got, want in (r["sg"], r["sg_root"]):
        for k, v in want.items():
            assert got[k].tobytes() == v.tobytes(), k
