"""The one-lane fused kernel (csrc/fs_arena1.h, k_step_n1) vs the CPU oracle.

fs_step_n launches with action rows run the one-lane kernel from 2 x 64 x SIMDs arenas on
(131 072 on MI355X) and the two-lane kernel below that; FOOTSIES_FUSED_LANES=1 / 2 forces one.
Here: the one-lane kernel at the size where it is selected (both P2 kinds with rows), every
float / auto-reset / reward mode and P2 kind at a small size, and the fused tests of
test_gpu_api.py re-run in a child process with the one-lane kernel forced."""
import os
import subprocess
import sys

import numpy as np
import pytest

from footsies_gym_amd import _abi
from tests.parity_utils import compare_outputs, compare_states

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P2 = {"external": _abi.FS_P2_EXTERNAL, "bot": _abi.FS_P2_BOT, "noop": _abi.FS_P2_NOOP}
FM = {"strict": _abi.FS_FLOAT_STRICT32, "double": _abi.FS_FLOAT_DOUBLE}
AR = {"same_step": _abi.FS_AUTORESET_SAME_STEP, "next_step": _abi.FS_AUTORESET_NEXT_STEP}


def fused_vs_oracle(oracle_lib, N, T, p2, fm="strict", ar="same_step", dense=True, seed=5, chunks=1):
    """`chunks` fs_step_n launches of T ticks with device action rows and a [T][N] trajectory;
    every row and the final hidden state against the oracle stepped tick by tick."""
    import torch
    from footsies_gym_amd.simulator import FootsiesSim
    sim = FootsiesSim(N, p2_mode=p2, float_mode=fm, autoreset_mode=ar, dense_reward=dense, seed=seed)
    ora = oracle_lib.Oracle(N, p2_mode=P2[p2], float_mode=FM[fm], autoreset_mode=AR[ar], dense_reward=dense,
                            base_seed=seed)
    traj = sim.alloc_trajectory(T)
    for c in range(chunks):
        p1, p2a = sim.hash_actions(T, seed=0xA1 + c, t0=c * T, p2=p2 == "external")
        sim.step_n(T, p1, p2a if p2 == "external" else None, trajectory=traj)
        torch.cuda.synchronize()
        tr = {k: v.cpu().numpy() for k, v in traj.items()}
        h1 = p1.cpu().numpy()
        h2 = p2a.cpu().numpy() if p2 == "external" else None
        for t in range(T):
            exp = ora.step(h1[t], None if h2 is None else h2[t])
            compare_outputs(exp, {k: v[t] for k, v in tr.items()}, step=c * T + t, same_step=ar == "same_step")
        compare_states(ora.state(), sim.get_state(), step=(c + 1) * T - 1)
    sim.close()


@pytest.mark.parametrize("p2", ["external", "bot"])
def test_one_lane_kernel_at_its_size(oracle_lib, p2):
    """131 072 arenas: the size from which fs_step_n selects the one-lane kernel (two of its
    waves per SIMD); two launches of 40 ticks, an odd-length one after an even one."""
    if os.environ.get("FOOTSIES_FUSED_LANES") == "2":
        pytest.skip("the two-lane kernel is forced")
    fused_vs_oracle(oracle_lib, 131072, 40, p2, chunks=1)
    fused_vs_oracle(oracle_lib, 131072, 41, p2, seed=6)


def packed_vs_oracle(oracle_lib, N, launches, p2, seed=5):
    """fs_step_n_packed launches of the given tick counts over device rows into one packed
    trajectory; every record of every launch (unpacked) and the final state against the oracle."""
    import torch
    from footsies_gym_amd._lib import lib
    from footsies_gym_amd.simulator import FootsiesSim, unpack_trajectory
    sim = FootsiesSim(N, p2_mode=p2, seed=seed)
    ora = oracle_lib.Oracle(N, p2_mode=P2[p2], base_seed=seed)
    ext = p2 == "external"
    traj = sim.alloc_packed_trajectory(max(launches))
    k = 0
    for c, T in enumerate(launches):
        p1, p2a = sim.hash_actions(T, seed=0xB7, t0=k, p2=ext)
        sim.step_n_packed(T, p1, p2a if ext else None, trajectory=traj)
        torch.cuda.synchronize()
        h1, h2 = p1.cpu().numpy(), (p2a.cpu().numpy() if ext else None)
        for t in range(T):
            exp = ora.step(h1[t], None if h2 is None else h2[t])
            rec = {key: (None if v is None else v[t].cpu().numpy()) for key, v in traj.items()}
            compare_outputs(exp, {key: np.ascontiguousarray(v) for key, v in unpack_trajectory(rec).items()}, step=k + t)
        k += T
    compare_states(ora.state(), sim.get_state(), step=k)
    name = lib().fs_step_kernel(sim.handle, max(launches), _abi.FS_KERNEL_PACKED).decode()
    sim.close()
    return name


@pytest.mark.parametrize("N", [131072, 262144])
@pytest.mark.parametrize("p2", ["external", "bot"])
def test_packed_kernel_at_c4_strong_scaling_sizes(oracle_lib, N, p2):
    """fs_step_n_packed at C4's one- and two-GPU strong-scaling shapes (262 144 and 131 072 arenas
    per GPU): the one-lane packed kernel (k_step_n1_packed), except a remote P2's at 262 144, which
    runs the two-lane one (fs_kernels.hip fused_one_lane); its records against the oracle, an even
    launch then an odd one (the row pipeline's tail).  The forced runs (FOOTSIES_FUSED_LANES=1 / 2)
    hold the other kernel at the same sizes."""
    forced = os.environ.get("FOOTSIES_FUSED_LANES", "")
    name = packed_vs_oracle(oracle_lib, N, [24, 17], p2)
    one = forced == "1" or (not forced and not (N == 262144 and p2 == "external"))
    assert name == ("fsk::k_step_n1_packed<0, %d>" if one else "fsk::k_step_n_packed<0, %d>") % P2[p2], name


def test_c4_sizes_with_each_kernel_forced():
    """test_packed_kernel_at_c4_strong_scaling_sizes in child processes with the one-lane and the
    two-lane kernel forced: both kernels against the oracle at 131 072 and 262 144 arenas, remote P2
    and bot."""
    if os.environ.get("FOOTSIES_FUSED_LANES"):
        pytest.skip("already the child")
    for lanes in ("1", "2"):
        env = dict(os.environ, FOOTSIES_FUSED_LANES=lanes)
        r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "gpu", "-p", "no:cacheprovider",
                            os.path.join(ROOT, "tests", "test_gpu_one_lane.py") + "::test_packed_kernel_at_c4_strong_scaling_sizes"],
                           cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, lanes + r.stdout[-4000:] + r.stderr[-2000:]
        assert "4 passed" in r.stdout, r.stdout[-2000:]


@pytest.mark.parametrize("p2", ["external", "bot", "noop"])
@pytest.mark.parametrize("fm,ar,dense", [("strict", "same_step", True), ("double", "same_step", True),
                                         ("strict", "next_step", True), ("double", "next_step", False),
                                         ("strict", "same_step", False)])
def test_modes_fused(oracle_lib, p2, fm, ar, dense):
    """Every float model, auto-reset mode and reward kind with each P2, fused with rows at a
    small size (whichever kernel the environment selects: the two-lane one by default here, the
    one-lane one in the child process below)."""
    fused_vs_oracle(oracle_lib, 3001, 97, p2, fm, ar, dense, seed=7, chunks=2)


def test_fused_tests_with_the_one_lane_kernel_forced():
    """This file's mode tests, test_gpu_api.py's fused tests (trajectory vs single steps,
    ragged 1 / 33 / 97-arena grids and odd tick counts, frame_delay, launches split by the
    32-bit offset limit) and test_gpu_packed.py's packed-vs-per-field twins (so the one-lane
    packed kernel meets the one-lane per-field one on every mode) in one child process with
    FOOTSIES_FUSED_LANES=1."""
    if os.environ.get("FOOTSIES_FUSED_LANES"):
        pytest.skip("already the child")
    env = dict(os.environ, FOOTSIES_FUSED_LANES="1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "gpu", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_gpu_one_lane.py") + "::test_modes_fused",
                        os.path.join(ROOT, "tests", "test_gpu_api.py"), os.path.join(ROOT, "tests", "test_gpu_packed.py"),
                        "-k", "test_modes_fused or step_n_trajectory or fused_ragged or frame_delay_paths or long_fused "
                              "or packed_trajectory"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert " passed" in r.stdout and " failed" not in r.stdout, r.stdout[-2000:]
