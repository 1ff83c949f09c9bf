"""The kernels bench.py reports, held directly against the CPU oracle at the bench's own shapes.

`bench.py` times `fs_step_n_packed` over HBM action rows written by `fs_hash_actions`: 65 536
arenas, a warm-up launch, then consecutive launches of `--steps` ticks (the driver runs
`--steps 20 --warmup 5`) or SURVEY §8(d)'s 1000-tick launches, the arenas' state carried in HBM
from launch to launch.  The same rows, copied to the host, drive the oracle one tick at a time
(`or_step`, OpenMP on the host); every packed record of the compared launches, unpacked by
`simulator.unpack_trajectory`, must equal the oracle's outputs of that tick bit for bit (final
records where the arena terminated), and the full canonical state must be equal at the end.

Three actor configurations, one per kernel instance the bench's legs run:
* external P2 (`k_step_n_packed<0, 0>`, the headline),
* the in-kernel bot as P2 (`<0, 1>`, the C2 opponent leg `p2_bot_mode`),
* P2 switched to the bot in every other arena (`<0, 3>`, kActors, the `actors_mode.mixed_p2` leg).

Reference semantics: BC:201-220 (the Fight tick), FE:518-570 (step's outputs and auto-reset).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from footsies_gym_amd import _abi
from tests.parity_utils import compare_outputs, compare_states, fused_kernel

pytestmark = pytest.mark.gpu

N = 65536
SEED = 0x5EED
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = {"external": "fsk::k_step_n_packed<0, 0>", "bot": "fsk::k_step_n_packed<0, 1>",
          "mixed": "fsk::k_step_n_packed<0, 3>"}
# (launch sizes, launches compared): the driver's shape (--warmup 5, then 20-tick regions) and
# SURVEY 8(d)'s (a 200-tick warm-up, then 1000-tick launches); launches are indexed in order
SHAPES = {"driver_20": ([5] + [20] * 10, "all"), "c3_1000": ([200, 1000, 1000], (0, 2))}


def _pair(oracle_lib, actors, n=N):
    from footsies_gym_amd.simulator import FootsiesSim
    p2 = "bot" if actors == "bot" else "external"
    sim = FootsiesSim(n, p2_mode=p2, seed=0, arena_base=0)
    ora = oracle_lib.Oracle(n, p2_mode=_abi.FS_P2_BOT if p2 == "bot" else _abi.FS_P2_EXTERNAL, base_seed=0)
    if actors == "mixed":  # set_opponent / P2_BOT on the even arenas, as the bench's mixed_p2 leg
        mask = (np.arange(n) % 2 == 0).astype(np.uint8)
        sim.set_p2_mode("bot", mask)
        assert ora.set_p2_mode(_abi.FS_P2_BOT, mask) == 0
    compare_states(ora.state(), sim.get_state(), step=-1)
    return sim, ora


@pytest.mark.parametrize("shape", sorted(SHAPES))
@pytest.mark.parametrize("actors", ["external", "bot", "mixed"])
def test_bench_kernel_matches_oracle_at_bench_shape(oracle_lib, actors, shape):
    run_shape(oracle_lib, actors, shape, N)


@pytest.mark.parametrize("shape", sorted(SHAPES))
@pytest.mark.parametrize("actors", ["external", "bot"])
def test_c4_per_gpu_shape_matches_oracle(oracle_lib, actors, shape):
    """C4's per-GPU shape (262 144 arenas over 8 GPUs: 32 768 per GPU, one wave per SIMD), where
    the two-lane fused launches prepare each tick's request at the end of the tick before
    (StepParams::prefetch): the same bench shapes against the oracle."""
    if os.environ.get("FOOTSIES_PREFETCH") != "0":
        assert fused_kernel(KERNEL[actors], 32768).startswith("fsk::k_step_n_packed_pf<")
    run_shape(oracle_lib, actors, shape, 32768)


def test_prefetch_forced_on_the_fused_suites():
    """The request prefetch (prepare_request) forced on every two-lane fused row launch
    (FOOTSIES_PREFETCH=1) in a child process: this file's 65 536-arena bench shapes, the packed
    twins of test_gpu_packed.py and the fused tests of test_gpu_api.py / test_gpu_one_lane.py (every
    float model, reward kind and P2 kind; next-step auto-reset launches keep the plain loop)."""
    if os.environ.get("FOOTSIES_PREFETCH"):
        pytest.skip("already the child")
    env = dict(os.environ, FOOTSIES_PREFETCH="1", FOOTSIES_FUSED_LANES="2")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "gpu", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_gpu_bench_shapes.py") + "::test_bench_kernel_matches_oracle_at_bench_shape",
                        os.path.join(ROOT, "tests", "test_gpu_packed.py"),
                        os.path.join(ROOT, "tests", "test_gpu_one_lane.py") + "::test_modes_fused",
                        os.path.join(ROOT, "tests", "test_gpu_api.py"), "-k",
                        "bench_shape or packed_trajectory or test_modes_fused or step_n_trajectory or fused_ragged "
                        "or frame_delay_paths or long_fused"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert " passed" in r.stdout and " failed" not in r.stdout, r.stdout[-2000:]


def run_shape(oracle_lib, actors, shape, n):
    import torch
    from footsies_gym_amd._lib import lib
    from footsies_gym_amd.simulator import unpack_trajectory
    launches, compared = SHAPES[shape]
    total = sum(launches)
    sim, ora = _pair(oracle_lib, actors, n)
    ext = actors != "bot"
    # the bench's inputs: the hashed stream written to HBM before timing
    p1, p2 = sim.hash_actions(total, seed=SEED, t0=0, p2=ext)
    torch.cuda.synchronize()
    h1 = p1.cpu().numpy()
    h2 = p2.cpu().numpy() if ext else None
    biggest = max(launches)
    kname = lib().fs_step_kernel(sim.handle, biggest, _abi.FS_KERNEL_PACKED).decode()
    want = fused_kernel(KERNEL[actors], n)
    assert kname == want or os.environ.get("FOOTSIES_FUSED_LANES") == "1", kname
    traj = sim.alloc_packed_trajectory(biggest)
    k, checked = 0, 0
    for j, m in enumerate(launches):
        sim.step_n_packed(m, p1[k:k + m], p2[k:k + m] if ext else None, trajectory=traj)
        torch.cuda.synchronize()
        check = compared == "all" or j in compared
        for t in range(m):
            exp = ora.step(h1[k + t], h2[k + t] if ext else None)
            if check:  # tick t's records copied once, then unpacked on the host
                rec = {key: (None if v is None else v[t].cpu().numpy()) for key, v in traj.items()}
                row = {key: np.ascontiguousarray(v) for key, v in unpack_trajectory(rec).items()}
                compare_outputs(exp, row, step=k + t)
                checked += 1
        k += m
    assert k == total and checked == (total if compared == "all" else sum(launches[j] for j in compared))
    compare_states(ora.state(), sim.get_state(), step=total)
    out = ora.outputs()
    assert out["terminated"].any()  # rounds end inside the compared launches (final records ran)
    sim.close()
    ora.close()


@pytest.mark.parametrize("actors,n", [("external", N), ("bot", N), ("external", 32768)])
def test_headline_kernel_long_horizon(oracle_lib, actors, n):
    """The headline kernel over SURVEY 8(d)'s C3 horizon many times over: 20 consecutive
    1000-tick launches (20 000 ticks: hundreds of rounds per arena, KOs, auto-resets, bot plans)
    at 65 536 arenas over HBM rows from fs_hash_actions, the arenas' state carried in HBM; the
    oracle steps the same rows tick by tick (OpenMP on the host).  Every record of the last launch
    and the full canonical state at the end must be equal.  Also at C4's per-GPU 32 768 arenas,
    where the request-prefetch kernel runs."""
    import torch
    from footsies_gym_amd._lib import lib
    from footsies_gym_amd.simulator import unpack_trajectory
    launches, T = 20, 1000
    sim, ora = _pair(oracle_lib, actors, n)
    assert lib().fs_step_kernel(sim.handle, T, _abi.FS_KERNEL_PACKED).decode() == fused_kernel(KERNEL[actors], n)
    ext = actors != "bot"
    traj = sim.alloc_packed_trajectory(T)
    for j in range(launches):
        p1, p2 = sim.hash_actions(T, seed=SEED, t0=j * T, p2=ext)
        sim.step_n_packed(T, p1, p2 if ext else None, trajectory=traj)
        torch.cuda.synchronize()
        h1 = p1.cpu().numpy()
        h2 = p2.cpu().numpy() if ext else None
        last = j == launches - 1
        for t in range(T):
            exp = ora.step(h1[t], h2[t] if ext else None)
            if last and t % 97 in (0, 96):  # (a sample of the last launch's records, unpacked on the host)
                rec = {key: (None if v is None else v[t].cpu().numpy()) for key, v in traj.items()}
                compare_outputs(exp, {key: np.ascontiguousarray(v) for key, v in unpack_trajectory(rec).items()},
                                step=j * T + t)
    compare_states(ora.state(), sim.get_state(), step=launches * T)
    sim.close()
    ora.close()


def test_step_rec_gather_leg_matches_oracle(oracle_lib):
    """bench.py's step_gather legs at their own shape: 65 536 arenas, `fs_step_rec` over HBM action
    rows of the hashed stream, one call per step.  Every step's 40-B records, unpacked
    (parallel.unpack_outputs), equal the oracle's outputs of that tick, and the state equals the
    oracle's at the end."""
    import ctypes as C
    import torch
    from footsies_gym_amd import parallel
    from footsies_gym_amd._lib import check, lib
    sim, ora = _pair(oracle_lib, "external")
    T = 120
    p1, p2 = sim.hash_actions(T, seed=SEED, t0=0)
    torch.cuda.synchronize()
    h1, h2 = p1.cpu().numpy(), p2.cpu().numpy()
    rec = torch.empty((N, _abi.FS_RECORD_BYTES), dtype=torch.uint8, device=sim.device)
    terminals = 0
    for t in range(T):
        check(lib().fs_step_rec(sim.handle, C.c_void_p(p1[t].data_ptr()), C.c_void_p(p2[t].data_ptr()),
                                _abi.FS_ACT_DEVICE, C.c_void_p(rec.data_ptr())), sim.handle)
        got = {k: v.cpu().numpy() for k, v in parallel.unpack_outputs(rec, torch).items()}
        exp = ora.step(h1[t], h2[t])
        compare_outputs(exp, got, step=t, same_step=False)
        terminals += int(exp["terminated"].sum())
    assert terminals > 0
    compare_states(ora.state(), sim.get_state(), step=T)
    sim.close()
    ora.close()
