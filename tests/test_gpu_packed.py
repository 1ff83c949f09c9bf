"""fs_step_n_packed: the fused row loop writing packed trajectory records (16 B per lane plus the
f64 reward, include/footsies.h fs_packed_traj) instead of one array per field.  Every field, read
through simulator.unpack_trajectory's strided views, must equal the fs_step_n trajectory of a twin
handle on the same state and actions, byte for byte (the per-field path is itself held to the
oracle by test_gpu_parity / test_gpu_api), and the two handles must end in the same state."""
import os

import numpy as np
import pytest

from footsies_gym_amd import _abi
from tests.parity_utils import compare_states, fused_kernel, random_states

pytestmark = pytest.mark.gpu


def _twins(n, p2, autoreset="same_step", seed=5, states=None):
    from footsies_gym_amd.simulator import FootsiesSim
    a = FootsiesSim(n, p2_mode=p2, seed=seed, autoreset_mode=autoreset)
    b = FootsiesSim(n, p2_mode=p2, seed=seed, autoreset_mode=autoreset)
    if states is not None:
        a.set_state(states)
        b.set_state(states)
    return a, b


def _compare(a, b, T, p1, p2):
    import torch
    from footsies_gym_amd.simulator import unpack_trajectory
    traj = a.alloc_trajectory(T)
    a.step_n(T, p1, p2, trajectory=traj)
    pk = b.step_n_packed(T, p1, p2)
    torch.cuda.synchronize()
    got = {k: np.ascontiguousarray(v.cpu().numpy()) for k, v in unpack_trajectory(pk).items()}
    exp = {k: v.cpu().numpy() for k, v in traj.items()}
    assert set(got) <= set(exp), sorted(set(got) - set(exp))
    for k, e in exp.items():
        if k not in got:  # (next-step auto-reset: neither layout has final records)
            assert k.startswith("final_") and not e.any(), k
            continue
        g = got[k]
        assert g.dtype == e.dtype and g.shape == e.shape, (k, g.dtype, e.dtype, g.shape, e.shape)
        # byte for byte (floats by their bits)
        bad = np.argwhere((g.view(np.uint8).reshape(g.shape + (-1,)) != e.view(np.uint8).reshape(e.shape + (-1,))).any(-1))
        assert bad.size == 0, "%s differs first at %s: packed %r, per-field %r" % (
            k, bad[0], g[tuple(bad[0])], e[tuple(bad[0])])
    # the pad bytes of P2's record (14, 15) and P2's word 3 of a final record stay zero
    lanes = pk["lanes"].cpu().numpy()
    assert not lanes[:, :, 1, 14:].any()
    if pk["final_lanes"] is not None:
        assert not pk["final_lanes"].cpu().numpy()[:, :, 1, 12:].any()
    compare_states(a.get_state(), b.get_state())
    return exp


@pytest.mark.parametrize("n,T,p2,autoreset", [(4096, 301, "external", "same_step"), (1000, 200, "bot", "same_step"),
                                              (777, 150, "noop", "next_step"), (97, 1, "external", "same_step"),
                                              (33, 64, "bot", "next_step")])
def test_packed_trajectory_equals_per_field(n, T, p2, autoreset):
    """Same-step and next-step auto-reset, every fixed P2 mode, ragged grids, odd tick counts (the
    loop's tail) and one tick; enough ticks that rounds end (final records) in the larger runs."""
    a, b = _twins(n, p2, autoreset)
    p1, q2 = a.hash_actions(T, seed=0x77, p2=p2 == "external")
    exp = _compare(a, b, T, p1, q2 if p2 == "external" else None)
    if n >= 1000:
        assert exp["terminated"].any()


def test_packed_trajectory_per_arena_actors_and_general_geometry():
    """Loaded arbitrary states with P2 switched to the bot in some arenas (the kActors kernel) and
    fighters off the ground / facing the other way (the general-geometry tick)."""
    rng = np.random.default_rng(41)
    st = random_states(2048, rng, p2="external", p2_bot_frac=0.3, geom_frac=0.3)
    a, b = _twins(2048, "external", states=st)
    p1, q2 = a.hash_actions(120, seed=0x99)
    _compare(a, b, 120, p1, q2)


def test_packed_trajectory_split_launches(monkeypatch):
    """A call split into several launches over row ranges (FOOTSIES_MAX_LAUNCH_ROWS, the test hook of
    the 32-bit offset limit) writes the same records as one launch."""
    monkeypatch.setenv("FOOTSIES_MAX_LAUNCH_ROWS", str(3 * 500 + 7))
    a, b = _twins(500, "external")
    p1, q2 = a.hash_actions(40, seed=0x55)
    _compare(a, b, 40, p1, q2)


def test_packed_trajectory_full_size():
    """C3's size: 65 536 arenas, 60 ticks."""
    a, b = _twins(65536, "external", seed=9)
    p1, q2 = a.hash_actions(60, seed=0x5EED)
    _compare(a, b, 60, p1, q2)


def test_packed_trajectory_argument_errors():
    import torch
    from footsies_gym_amd._lib import FootsiesError
    from footsies_gym_amd.simulator import FootsiesSim
    sim = FootsiesSim(64, p2_mode="external")
    p1, q2 = sim.hash_actions(4, seed=1)
    traj = sim.alloc_packed_trajectory(4)
    with pytest.raises(FootsiesError):  # same-step auto-reset needs the final records
        sim.step_n_packed(4, p1, q2, trajectory=dict(traj, final_lanes=None))
    with pytest.raises(ValueError):  # a non-contiguous buffer
        sim.step_n_packed(4, p1, q2, trajectory=dict(traj, lanes=traj["lanes"].transpose(0, 1)))
    # buffers the kernels would address raw are checked first: host, short or mistyped ones
    with pytest.raises(ValueError):
        sim.step_n_packed(4, p1.cpu(), q2, trajectory=traj)
    with pytest.raises(ValueError):
        sim.step_n_packed(4, p1[:2], q2, trajectory=traj)
    with pytest.raises(ValueError):
        sim.step_n(4, p1, q2.to(torch.int32))
    with pytest.raises(ValueError):
        sim.step_n(4, p1, q2, trajectory=dict(sim.alloc_trajectory(2)))
    delayed = FootsiesSim(64, p2_mode="external", frame_delay=2)
    with pytest.raises(FootsiesError):  # the delayed queue reads the per-field outputs
        delayed.step_n_packed(4, p1, q2)
    from footsies_gym_amd._lib import lib  # the kernel a packed call runs, as rocprofv3 names it
    one = os.environ.get("FOOTSIES_FUSED_LANES") == "1"  # (test_gpu_one_lane.py's child forces the one-lane kernel)
    assert lib().fs_step_kernel(sim.handle, 4, _abi.FS_KERNEL_PACKED).decode() == (
        "fsk::k_step_n1_packed<0, 0>" if one else fused_kernel("fsk::k_step_n_packed<0, 0>", 64))
    torch.cuda.synchronize()


@pytest.mark.parametrize("dense", [True, False])
def test_packed_trajectory_double_float_mode_and_sparse_reward(dense):
    """The binary64-temporaries float model (FS_FLOAT_DOUBLE: the <1, P2> kernel instances) and
    the sparse reward."""
    from footsies_gym_amd.simulator import FootsiesSim
    a = FootsiesSim(2000, p2_mode="external", seed=21, float_mode="double", dense_reward=dense)
    b = FootsiesSim(2000, p2_mode="external", seed=21, float_mode="double", dense_reward=dense)
    p1, q2 = a.hash_actions(200, seed=0x42)
    exp = _compare(a, b, 200, p1, q2)
    assert exp["terminated"].any()


def test_packed_trajectory_by_example():
    """by_example (the bot plays P1 as well as P2: the kActors kernel with P1's rows unread)."""
    from footsies_gym_amd.simulator import FootsiesSim
    a = FootsiesSim(1500, p2_mode="bot", p1_mode="bot", seed=12)
    b = FootsiesSim(1500, p2_mode="bot", p1_mode="bot", seed=12)
    p1, _ = a.hash_actions(150, seed=0x31, p2=False)
    _compare(a, b, 150, p1, None)
