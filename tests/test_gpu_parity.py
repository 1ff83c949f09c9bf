"""HIP path (libfootsies.so through FootsiesSim) vs the CPU oracle, in lockstep.

Bit-exact on every output and on the canonical hidden state (fs_get_state).
"""
import numpy as np
import pytest

from footsies_gym_amd import _abi
from tests.parity_utils import compare_outputs, compare_states, random_states

pytestmark = pytest.mark.gpu

P2 = {"external": _abi.FS_P2_EXTERNAL, "bot": _abi.FS_P2_BOT, "noop": _abi.FS_P2_NOOP}
FM = {"strict": _abi.FS_FLOAT_STRICT32, "double": _abi.FS_FLOAT_DOUBLE}
AR = {"same_step": _abi.FS_AUTORESET_SAME_STEP, "next_step": _abi.FS_AUTORESET_NEXT_STEP}


def make_pair(oracle_lib, n, p2, fm="strict", ar="same_step", dense=True, seed=0):
    from footsies_gym_amd.simulator import FootsiesSim
    sim = FootsiesSim(n, p2_mode=p2, float_mode=fm, autoreset_mode=ar, dense_reward=dense, seed=seed)
    ora = oracle_lib.Oracle(n, p2_mode=P2[p2], float_mode=FM[fm], autoreset_mode=AR[ar], dense_reward=dense,
                            base_seed=seed)
    return sim, ora


def run_lockstep(sim, ora, steps, rng, state_every=50, sticky=0.0):
    n = sim.num_envs
    compare_outputs(ora.outputs(), sim.outputs_numpy(), step=-1)
    compare_states(ora.state(), sim.get_state(), step=-1)
    a1 = rng.integers(0, 8, n).astype(np.uint8)
    a2 = rng.integers(0, 8, n).astype(np.uint8)
    for t in range(steps):
        # sticky random actions exercise holds (charge specials), dashes and walks
        keep = rng.random(n) < sticky
        a1 = np.where(keep, a1, rng.integers(0, 8, n)).astype(np.uint8)
        keep = rng.random(n) < sticky
        a2 = np.where(keep, a2, rng.integers(0, 8, n)).astype(np.uint8)
        eo = ora.step(a1, a2 if sim.p2_mode == "external" else None)
        go = sim.step(a1, a2 if sim.p2_mode == "external" else None)
        go = sim.outputs_numpy()
        compare_outputs(eo, go, step=t, same_step=sim.autoreset_mode == "same_step")
        if state_every and (t % state_every == 0 or t == steps - 1):
            compare_states(ora.state(), sim.get_state(), step=t)


@pytest.mark.parametrize("p2", ["external", "bot", "noop"])
def test_lockstep_random(oracle_lib, p2):
    sim, ora = make_pair(oracle_lib, 512, p2, seed=11)
    run_lockstep(sim, ora, 600, np.random.default_rng(1), sticky=0.0)


@pytest.mark.parametrize("n", [1, 7, 32, 33])
@pytest.mark.parametrize("p2", ["external", "bot"])
def test_lockstep_few_arenas_host_actions(oracle_lib, n, p2):
    """Host actions of at most 32 arenas travel in the kernel arguments (no staging copy); 33
    takes the staging path.  Both lockstep with the oracle, terminals and resets included."""
    sim, ora = make_pair(oracle_lib, n, p2, seed=3 + n)
    run_lockstep(sim, ora, 2500, np.random.default_rng(n), state_every=250, sticky=0.5)


@pytest.mark.parametrize("p2", ["external", "bot"])
def test_lockstep_sticky(oracle_lib, p2):
    sim, ora = make_pair(oracle_lib, 512, p2, seed=5)
    run_lockstep(sim, ora, 800, np.random.default_rng(2), sticky=0.9)


@pytest.mark.parametrize("fm,ar,dense", [("double", "same_step", True), ("strict", "next_step", True),
                                          ("strict", "same_step", False), ("double", "next_step", False)])
def test_lockstep_modes(oracle_lib, fm, ar, dense):
    sim, ora = make_pair(oracle_lib, 256, "bot", fm=fm, ar=ar, dense=dense, seed=3)
    run_lockstep(sim, ora, 500, np.random.default_rng(3), sticky=0.7)


def test_resets_lockstep(oracle_lib):
    sim, ora = make_pair(oracle_lib, 256, "bot", seed=9)
    rng = np.random.default_rng(4)
    for rnd in range(6):
        run_lockstep(sim, ora, 60, rng, state_every=20, sticky=0.5)
        mask = (rng.random(256) < 0.5).astype(np.uint8)
        seeds = rng.integers(0, 2**31, 256).astype(np.uint64) if rnd % 2 else None
        hard = rnd % 3 == 0
        seed_only = rnd == 4
        flags = (_abi.FS_RESET_SEED_ONLY if seed_only else _abi.FS_RESET_HARD if hard else _abi.FS_RESET_IF_NEEDED)
        if seed_only:
            seeds = rng.integers(0, 2**31, 256).astype(np.uint64)
        eo = ora.reset(seeds=seeds, mask=mask, flags=flags)
        sim.reset(seeds=seeds, mask=mask, hard=hard, seed_only=seed_only)
        compare_outputs(eo, sim.outputs_numpy(), step=-2)
        compare_states(ora.state(), sim.get_state(), step=-2)


def test_lockstep_4096_bot_long(oracle_lib):
    """Config 2 shape: 4096 arenas, random P1 vs scripted bot P2, 10k steps."""
    sim, ora = make_pair(oracle_lib, 4096, "bot", seed=0)
    run_lockstep(sim, ora, 10000, np.random.default_rng(123), state_every=500, sticky=0.5)


@pytest.mark.parametrize("p2", ["external", "bot", "noop"])
def test_lockstep_from_random_loaded_states(oracle_lib, p2):
    """STATE_LOAD of arbitrary states into both, then lockstep: the table-driven request chain,
    hit resolution and the bot's split queues agree with the oracle's restatement on the rare
    paths too (the oracle rebuilds the bot's real queues and FightState ring from the state)."""
    n = 4096
    sim, ora = make_pair(oracle_lib, n, p2, seed=21)
    st = random_states(n, np.random.default_rng(77), p2=p2)
    assert ora.set_state(st) == 0
    sim.set_state(st)
    compare_states(ora.state(), sim.get_state(), step=-1)
    run_lockstep(sim, ora, 200, np.random.default_rng(78), state_every=10, sticky=0.6)


# stage edges (±5), outside them, ±0.0 and the smallest denormals: the stage push applies -0.0
# (the exact identity of IEEE addition) when it does not push, and the character push's tie rule
EDGE_X = np.array([-0.0, 0.0, 1e-45, -1e-45, 0.3, -0.3, 4.5, -4.5, 4.99, -4.99, 5.0, -5.0, 5.5, -5.5, 7.0, -7.0],
                  dtype=np.float32)


@pytest.mark.parametrize("fm", ["strict", "double"])
def test_lockstep_edge_positions(oracle_lib, fm):
    """Loaded states with both fighters on edge positions (and 10 % of arenas on the same x),
    stepped in lockstep: positions and every other output bit-exact, ±0.0 included."""
    n = 2048
    sim, ora = make_pair(oracle_lib, n, "external", fm=fm, seed=31)
    rng = np.random.default_rng(91)
    st = random_states(n, rng)
    for k in range(2):
        st["f"][:, k]["position_x"] = rng.choice(EDGE_X, n)
    tie = rng.random(n) < 0.1
    st["f"][:, 1]["position_x"] = np.where(tie, st["f"][:, 0]["position_x"], st["f"][:, 1]["position_x"])
    assert np.signbit(st["f"]["position_x"]).any() and (st["f"]["position_x"] == 0).any()
    assert ora.set_state(st) == 0
    sim.set_state(st)
    compare_states(ora.state(), sim.get_state(), step=-1)
    run_lockstep(sim, ora, 120, np.random.default_rng(92), state_every=5, sticky=0.5)


@pytest.mark.parametrize("n_envs,ticks,p2", [(65536, 500, "external"), (262144, 200, "bot"), (262144, 200, "external")])
def test_full_size_fused_matches_oracle(oracle_lib, n_envs, ticks, p2):
    """BASELINE sizes (C3: 65 536 arenas; C4: 262 144 = 8 x 32 768 on one GPU): the fused kernel
    with in-kernel hashed actions, in chunks, against the oracle on the same hashed stream --
    every arena's full state and the last step's outputs bit-exact."""
    import torch
    from footsies_gym_amd.simulator import FootsiesSim
    p2m = {"external": _abi.FS_P2_EXTERNAL, "bot": _abi.FS_P2_BOT}[p2]
    sim = FootsiesSim(n_envs, p2_mode=p2, seed=17)
    ora = oracle_lib.Oracle(n_envs, p2_mode=p2m, base_seed=17)
    done = 0
    for chunk in (1, 99, ticks - 100):
        sim.step_n(chunk, None, None, action_seed=0xC3C4)
        ora.step_n_hashed(chunk, 0xC3C4)
        done += chunk
    torch.cuda.synchronize()
    assert done == ticks
    compare_states(ora.state(), sim.get_state())
    compare_outputs(ora.outputs(), sim.outputs_numpy())
    sim.close()
    ora.close()


@pytest.mark.parametrize("p2", ["external", "bot"])
def test_long_horizon_c3_size_matches_oracle(oracle_lib, p2):
    """C3's 65 536 arenas over 20 000 ticks (many rounds per arena: KOs, auto-resets, bot
    plans, recordings) in 20 fused launches of 1 000 ticks with in-kernel hashed actions: the full
    state of every arena and the last outputs equal the oracle's (OpenMP on the host)."""
    import torch
    from footsies_gym_amd.simulator import FootsiesSim
    n, launches, ticks = 65536, 20, 1000
    p2m = {"external": _abi.FS_P2_EXTERNAL, "bot": _abi.FS_P2_BOT}[p2]
    sim = FootsiesSim(n, p2_mode=p2, seed=23)
    ora = oracle_lib.Oracle(n, p2_mode=p2m, base_seed=23)
    for _ in range(launches):
        sim.step_n(ticks, None, None, action_seed=0x10C)
    ora.step_n_hashed(launches * ticks, 0x10C)
    torch.cuda.synchronize()
    compare_states(ora.state(), sim.get_state())
    compare_outputs(ora.outputs(), sim.outputs_numpy())
    sim.close()
    ora.close()


@pytest.mark.parametrize("p2,fm", [("external", "strict"), ("bot", "strict"), ("external", "double")])
def test_lockstep_general_geometry(oracle_lib, p2, fm):
    """STATE_LOAD of fighters off the ground (position.y != 0) and with flipped facings
    (Fighter.LoadState F:741-744; the game itself never produces either) runs the kernels'
    general-geometry tick -- box y extents from kRecY, y carried through both pushes (each push
    adds a fighter's y to itself, BC:491-498, 511-515), mirrored boxes, movement and input
    parsing -- against the oracle's direct restatement of the C#, one tick per launch, every
    output and the full state (y and facing included) bit-exact; a round start clears both."""
    n = 4096
    sim, ora = make_pair(oracle_lib, n, p2, fm=fm, seed=41)
    st = random_states(n, np.random.default_rng(141), p2=p2, geom_frac=0.3)
    assert (st["f"]["position_y"] != 0).any() and (st["f"]["facing_flipped"] == 1).any()
    assert ora.set_state(st) == 0
    sim.set_state(st)
    compare_states(ora.state(), sim.get_state(), step=-1)
    run_lockstep(sim, ora, 200, np.random.default_rng(142), state_every=5, sticky=0.5)
    end = sim.get_state()
    y0, y1 = st["f"]["position_y"], end["f"]["position_y"]
    moved = (y0 != 0) & (y1 != 0) & (y1 != y0)
    assert moved.any(), "no push carried a y"                      # the doubling quirk ran
    assert ((y0 != 0) & (y1 == 0)).any() and ((st["f"]["facing_flipped"] == 1) & (end["f"]["facing_flipped"] == 0)).any()


@pytest.mark.parametrize("p2", ["external", "bot"])
def test_fused_general_geometry_matches_oracle(oracle_lib, p2):
    """The fused kernel's general-geometry loop (fs_step_n after such a load; the two-lane kernel
    even where the one-lane one would run) against the oracle, every trajectory row and the final
    state; then the hashed-action loop on top."""
    import torch
    from footsies_gym_amd.simulator import FootsiesSim
    N, T = 2999, 120
    sim = FootsiesSim(N, p2_mode=p2, seed=7)
    ora = oracle_lib.Oracle(N, p2_mode=P2[p2], base_seed=7)
    st = random_states(N, np.random.default_rng(143), p2=p2, geom_frac=0.4)
    assert ora.set_state(st) == 0
    sim.set_state(st)
    p1, p2a = sim.hash_actions(T, seed=93, p2=p2 == "external")
    traj = sim.alloc_trajectory(T)
    sim.step_n(T, p1, p2a if p2 == "external" else None, trajectory=traj)
    torch.cuda.synchronize()
    tr = {k: v.cpu().numpy() for k, v in traj.items()}
    h1 = p1.cpu().numpy()
    h2 = p2a.cpu().numpy() if p2 == "external" else None
    for t in range(T):
        exp = ora.step(h1[t], None if h2 is None else h2[t])
        compare_outputs(exp, {k: v[t] for k, v in tr.items()}, step=t)
    compare_states(ora.state(), sim.get_state())
    sim.step_n(40, None, None, action_seed=0x6E0)
    ora.step_n_hashed(40, 0x6E0)
    torch.cuda.synchronize()
    compare_states(ora.state(), sim.get_state())
    compare_outputs(ora.outputs(), sim.outputs_numpy())


def test_standard_load_leaves_the_general_geometry_path():
    """fs_step_kernel names the kernel a launch runs: after a load with an airborne fighter the
    fused launch at >= 131 072 arenas takes the two-lane kernel (the one-lane one has no general-
    geometry tick); a later load of standard fighters only returns to the one-lane kernel."""
    import os
    from footsies_gym_amd._lib import lib
    from footsies_gym_amd.simulator import FootsiesSim
    if os.environ.get("FOOTSIES_FUSED_LANES"):
        pytest.skip("the kernel choice is forced")
    sim = FootsiesSim(131072, p2_mode="external", seed=3)
    name = lambda: lib().fs_step_kernel(sim.handle, 100, 0).decode()  # noqa: E731
    assert name() == "fsk::k_step_n1<0, 0>"
    st = sim.get_state()
    st["f"][5, 0]["position_y"] = np.float32(0.5)
    sim.set_state(st)
    assert name() == "fsk::k_step_n<0, 0>"
    # -0.0 is ground level for the boxes, but the pushes keep its sign and the round start writes
    # +0.0 (SetupBattleStart, F:120-135): only the general-geometry tick carries y
    st["f"][5, 0]["position_y"] = np.float32(-0.0)
    sim.set_state(st)
    assert name() == "fsk::k_step_n<0, 0>"
    st["f"][5, 0]["position_y"] = np.float32(0.0)
    sim.set_state(st)
    assert name() == "fsk::k_step_n1<0, 0>"
    st["f"][7, 1]["facing_flipped"] = 1
    sim.set_state(st)
    assert name() == "fsk::k_step_n<0, 0>"
    sim.close()
