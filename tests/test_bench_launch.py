"""bench.py's multi-rank launch on CPU: `python bench.py --gpus N` starts
N ranks itself (a torch.distributed.run child), each rank checks that the launcher's world size
is N, the regions are timed between barriers with the max over ranks, and rank 0 prints one
line whose value is the whole-job rate.  `--dry-run` replaces the simulator by a no-op CPU step,
so only the plumbing is exercised here; the GPU path is the same code after the step."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run_bench(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout,
                          env=env, cwd=ROOT)


def json_line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def check_c4_plan(out, gpus):
    """The c4_strong leg (BASELINE configs[3]) on every rank of the plain `bench.py --gpus N`:
    262 144 / N arenas per rank over contiguous global ranges, arena_base = rank x 262 144 / N."""
    c4 = out["c4_strong"]
    assert c4["global_envs"] == 262144 and c4["scaling"] == "strong"
    assert c4["envs_per_rank"] == [262144 // gpus] * gpus
    assert c4["arena_base_per_rank"] == [r * (262144 // gpus) for r in range(gpus)]
    assert sum(c4["envs_per_rank"]) == 262144


def test_c4_split():
    sys.path.insert(0, ROOT)
    import bench
    for world in (1, 2, 4, 8):
        shards = [bench.c4_split(world, r) for r in range(world)]
        assert [b for _, b in shards] == [r * 262144 // world for r in range(world)]
        assert all(n == 262144 // world for n, _ in shards)
        assert shards[-1][1] + shards[-1][0] == 262144
    assert bench.c4_split(3, 0) is None  # no even split: the leg is skipped


@pytest.mark.parametrize("gpus", [2, 3, 4])
def test_gpus_n_launches_n_ranks(gpus):
    p = run_bench(["--gpus", str(gpus), "--dry-run", "--dist-backend", "gloo", "--steps", "20", "--regions", "3",
                   "--envs", "1000"])
    assert p.returncode == 0, p.stderr[-2000:]
    out = json_line(p.stdout)
    assert out["dry_run"] is True
    assert out["n_gpus"] == gpus
    assert out["ranks"]["world_size"] == gpus and out["ranks"]["backend"] == "gloo"
    assert len(out["ranks"]["rank_walls_ms"]) == gpus
    assert out["config"]["global_envs"] == gpus * 1000
    if 262144 % gpus == 0:
        check_c4_plan(out, gpus)
    else:
        assert out["c4_strong"]["envs_per_rank"] == [0] * gpus
    # whole-job rate: every rank's arenas x steps over the max-over-ranks median region
    wall_s = out["ms_per_step"] * out["steps"] / 1e3
    assert out["value"] == pytest.approx(gpus * 1000 * out["steps"] / wall_s, rel=1e-9)
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in out


def test_single_rank_needs_no_launcher():
    p = run_bench(["--gpus", "1", "--dry-run", "--steps", "5", "--regions", "1"])
    assert p.returncode == 0, p.stderr[-2000:]
    out = json_line(p.stdout)
    assert out["n_gpus"] == 1 and out["ranks"]["world_size"] == 1
    check_c4_plan(out, 1)  # the curve's first point: all 262 144 arenas on one GPU


def test_world_size_must_match_gpus():
    """Under an outside launcher the rank refuses a --gpus that disagrees with WORLD_SIZE."""
    p = run_bench(["--gpus", "2", "--dry-run"], env_extra={"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "--gpus 2" in p.stderr and "3 rank" in p.stderr


def test_launch_command(monkeypatch):
    """The launcher is a torch.distributed.run child on 127.0.0.1 with one process per GPU,
    re-running bench.py with the same arguments."""
    sys.path.insert(0, ROOT)
    import bench
    seen = {}

    class R:
        returncode = 0

    def fake_run(cmd, env):
        seen["cmd"], seen["env"] = cmd, env
        return R()
    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "20"])
    assert bench.launch_ranks(bench.parse()) == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    assert cmd[-3:] == ["--gpus", "8", "--steps", "20"][-3:] and os.path.samefile(cmd[-5], BENCH)
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def test_eight_ranks_dry_run():
    """The driver's largest scaling point (N = 8) rehearsed on CPU: 8 gloo ranks, barriers, max over
    ranks, one line from rank 0 whose value is the whole-job rate."""
    p = run_bench(["--gpus", "8", "--dry-run", "--dist-backend", "gloo", "--steps", "10", "--regions", "3",
                   "--envs", "500"], timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json_line(p.stdout)
    assert out["n_gpus"] == 8 and out["ranks"]["world_size"] == 8 and len(out["ranks"]["rank_walls_ms"]) == 8
    assert out["config"]["global_envs"] == 8 * 500
    check_c4_plan(out, 8)
    wall_s = out["ms_per_step"] * out["steps"] / 1e3
    assert out["value"] == pytest.approx(8 * 500 * out["steps"] / wall_s, rel=1e-9)


def test_outside_launcher_without_gpus_flag():
    """`torchrun --nproc-per-node=2 bench.py` with no --gpus (advisor r03): the ranks take the
    launcher's world size instead of refusing it."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", "--master-port=%d" % port, BENCH, "--dry-run", "--dist-backend",
                        "gloo", "--steps", "5", "--regions", "2", "--envs", "100"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json_line(p.stdout)
    assert out["n_gpus"] == 2 and out["ranks"]["world_size"] == 2
