"""The actors on the HIP path vs the CPU oracle: P2 switched at runtime between the remote
actor and the bot (fs_set_p2_mode -- the P2_BOT command behind FootsiesEnv.set_opponent,
FE:458-480, BC:158-167) and the bot playing P1 (by_example, FE:230-232), through the per-arena
actor kernels (kActors).  Bit-exact on every output and the canonical state."""
import numpy as np
import pytest

from footsies_gym_amd import _abi
from tests import kat_actors
from tests.parity_utils import compare_outputs, compare_states, random_states
from tests.test_gpu_parity import AR, P2, run_lockstep

pytestmark = pytest.mark.gpu


def make_pair(oracle_lib, n, p2, p1="external", ar="same_step", seed=0, arena_base=0):
    from footsies_gym_amd.simulator import FootsiesSim
    sim = FootsiesSim(n, p2_mode=p2, p1_mode=p1, autoreset_mode=ar, seed=seed, arena_base=arena_base)
    ora = oracle_lib.Oracle(n, p2_mode=P2[p2], autoreset_mode=AR[ar], base_seed=seed, arena_base=arena_base,
                            p1_mode=_abi.FS_P1_BOT if p1 == "bot" else _abi.FS_P1_EXTERNAL)
    return sim, ora


@pytest.mark.parametrize("name", sorted(kat_actors.ALL))
def test_kat_actors_gpu(name):
    kat_actors.ALL[name](kat_actors.SimActors)


def test_kat_bot_plans_gpu():
    """The scripted bot's plan logic against the hand-derived restatement of BattleAI.cs
    (tests/kat_bot.py) through the HIP path: every distance bucket's draw size and outcome map at
    and around the bucket edges, the TwoHit rules that draw nothing, NoAttack at d > 4 still
    drawing, every index of every plan (FallBack2's forward "backward dash" included) for P2's bot
    and for P1's mirrored one, and the decision reading the previous call's FightState."""
    from tests import kat_bot
    kat_bot.run(lambda n, p1: kat_bot.SimBot(n, p1))


def switch_rounds(sim, ora, rng, rounds, steps, reset_every=0):
    """Lockstep in rounds; between rounds a random subset of arenas switches P2 to the bot and
    another back to the remote actor (mid-episode, pending bursts included), and every
    `reset_every` rounds a masked hard reset."""
    n = sim.num_envs
    for rnd in range(rounds):
        run_lockstep(sim, ora, steps, rng, state_every=steps // 2, sticky=0.5)
        for mode in (_abi.FS_P2_BOT, _abi.FS_P2_EXTERNAL):
            mask = (rng.random(n) < 0.3).astype(np.uint8)
            assert ora.set_p2_mode(mode, mask) == 0
            sim.set_p2_mode("bot" if mode == _abi.FS_P2_BOT else "external", mask)
        compare_states(ora.state(), sim.get_state(), step=-3)
        if reset_every and rnd % reset_every == reset_every - 1:
            mask = (rng.random(n) < 0.5).astype(np.uint8)
            eo = ora.reset(mask=mask, flags=_abi.FS_RESET_HARD)
            sim.reset(mask=mask, hard=True)
            compare_outputs(eo, sim.outputs_numpy(), step=-2)
            compare_states(ora.state(), sim.get_state(), step=-2)


@pytest.mark.parametrize("ar", ["same_step", "next_step"])
def test_lockstep_p2_switching(oracle_lib, ar):
    """4096 arenas, P2 toggled between remote and bot for random subsets every 40 steps over
    1200 steps, with masked RESETs: the never-Reset switched-in bot, its stale input and the
    remote actor's stale input through Intro ticks."""
    sim, ora = make_pair(oracle_lib, 4096, "external", ar=ar, seed=41)
    switch_rounds(sim, ora, np.random.default_rng(7), 30, 40, reset_every=4)


@pytest.mark.parametrize("p2", ["bot", "external", "noop"])
def test_lockstep_by_example(oracle_lib, p2):
    """P1 = the bot (by_example) against every P2 (for a remote P2, with switching): the two bots
    share one RNG, P1 drawing first."""
    sim, ora = make_pair(oracle_lib, 4096, p2, p1="bot", seed=5)
    rng = np.random.default_rng(8)
    if p2 == "external":
        switch_rounds(sim, ora, rng, 20, 50, reset_every=5)
    else:
        run_lockstep(sim, ora, 1000, rng, state_every=100, sticky=0.5)


@pytest.mark.parametrize("p1", ["external", "bot"])
def test_lockstep_actors_from_random_states(oracle_lib, p1):
    """Arbitrary loaded states with 30 % of the arenas' P2 switched to a bot that may or may not
    be ready, arbitrary queues for both bots, arbitrary stored inputs."""
    n = 4096
    sim, ora = make_pair(oracle_lib, n, "external", p1=p1, seed=12)
    st = random_states(n, np.random.default_rng(13), p2="external", p2_bot_frac=0.3)
    assert ora.set_state(st) == 0
    sim.set_state(st)
    compare_states(ora.state(), sim.get_state(), step=-1)
    run_lockstep(sim, ora, 200, np.random.default_rng(14), state_every=10, sticky=0.6)


@pytest.mark.parametrize("p1,hashed", [("external", False), ("external", True), ("bot", False), ("bot", True)])
def test_fused_actors_match_oracle(oracle_lib, p1, hashed):
    """fs_step_n (trajectory, or in-kernel hashed actions) through the actor kernels, a sharded
    arena_base included, against the oracle step by step."""
    import torch
    N, T, base = 2000, 300, 12345
    sim, ora = make_pair(oracle_lib, N, "external", p1=p1, seed=3, arena_base=base)
    mask = (np.arange(N) % 3 == 0).astype(np.uint8)
    assert ora.set_p2_mode(_abi.FS_P2_BOT, mask) == 0
    sim.set_p2_mode("bot", mask)
    if hashed:
        sim.step_n(T, None, None, action_seed=0xACE)
        ora.step_n_hashed(T, 0xACE)
        torch.cuda.synchronize()
        compare_outputs(ora.outputs(), sim.outputs_numpy())
    else:
        p1a, p2a = sim.hash_actions(T, seed=77)
        traj = sim.alloc_trajectory(T)
        sim.step_n(T, None if p1 == "bot" else p1a, p2a, trajectory=traj)
        torch.cuda.synchronize()
        tr = {k: v.cpu().numpy() for k, v in traj.items()}
        h1, h2 = p1a.cpu().numpy(), p2a.cpu().numpy()
        for t in range(T):
            exp = ora.step(h1[t], h2[t])
            compare_outputs(exp, {k: v[t] for k, v in tr.items()}, step=t)
    compare_states(ora.state(), sim.get_state())


def test_set_p2_mode_rejected_without_remote_p2():
    from footsies_gym_amd._lib import FootsiesError
    from footsies_gym_amd.simulator import FootsiesSim
    for p2 in ("bot", "noop"):
        sim = FootsiesSim(8, p2_mode=p2)
        with pytest.raises(FootsiesError):
            sim.set_p2_mode("bot")
        sim.close()


def test_vector_env_set_opponent_matches_oracle(oracle_lib):
    """FootsiesVectorEnv.set_opponent: the callable's arenas and the bot's, switched by mask and
    for all arenas, equal the oracle fed the same actions and P2_BOT commands; the single-env
    FootsiesEnv.set_opponent returns None and needs a custom opponent (FE:468-470)."""
    from footsies_gym_amd.vector_env import FootsiesEnv, FootsiesVectorEnv
    n = 512
    rng = np.random.default_rng(3)
    acts = {}

    def opp(obs, info):
        acts["p2"] = rng.integers(0, 8, n).astype(np.uint8)
        return acts["p2"]
    env = FootsiesVectorEnv(n, opponent=opp, seed=4, autoreset_mode="same_step")
    ora = oracle_lib.Oracle(n, p2_mode=_abi.FS_P2_EXTERNAL, base_seed=4)
    env.reset()
    plan = {20: (None, rng.random(n) < 0.5), 60: (opp, None), 90: (None, None), 150: (opp, rng.random(n) < 0.3)}
    bot = np.zeros(n, bool)
    for t in range(200):
        if t in plan:
            o, m = plan[t]
            assert env.set_opponent(o, mask=m) is None
            sel = np.ones(n, bool) if m is None else m
            change = sel & (~bot if o is None else bot)
            if change.any():
                ora.set_p2_mode(_abi.FS_P2_BOT if o is None else _abi.FS_P2_EXTERNAL, change.astype(np.uint8))
            bot = (bot | sel) if o is None else (bot & ~sel)
        a1 = rng.integers(0, 8, n).astype(np.uint8)
        acts["p2"] = np.zeros(n, np.uint8)
        obs, rew, term, trunc, info = env.step(a1)
        exp = ora.step(a1, acts["p2"])
        np.testing.assert_array_equal(rew.view(np.uint64), exp["reward"].view(np.uint64))
        np.testing.assert_array_equal(obs["move"], exp["move"])
        np.testing.assert_array_equal(obs["position"].view(np.uint32), exp["position"].view(np.uint32))
    compare_states(ora.state(), env.save_battle_state())
    env.close()
    single = FootsiesEnv(opponent=lambda o, i: (False, True, False))
    single.reset()
    assert single.set_opponent(None) is None
    single.step((True, False, False))
    assert single.set_opponent(lambda o, i: (True, False, True)) is None
    single.step((False, False, True))
    single.close()
    with pytest.raises(RuntimeError):
        FootsiesEnv().set_opponent(None)


def test_vector_env_by_example_ignores_actions(oracle_lib):
    """by_example: the agent's actions are not sent (FE:522-523); the bot plays P1."""
    from footsies_gym_amd.vector_env import FootsiesVectorEnv
    n = 256
    env = FootsiesVectorEnv(n, by_example=True, seed=6)
    ora = oracle_lib.Oracle(n, p2_mode=_abi.FS_P2_BOT, p1_mode=_abi.FS_P1_BOT, base_seed=6)
    env.reset()
    rng = np.random.default_rng(0)
    for t in range(300):
        obs, rew, term, trunc, info = env.step(rng.integers(0, 8, n))
        exp = ora.step(None)
        np.testing.assert_array_equal(info["p1_action"], np.stack([(exp["action"][:, 0] >> b) & 1 for b in range(3)],
                                                                  axis=-1).astype(bool))
        np.testing.assert_array_equal(rew.view(np.uint64), exp["reward"].view(np.uint64))
    compare_states(ora.state(), env.save_battle_state())
    env.close()
