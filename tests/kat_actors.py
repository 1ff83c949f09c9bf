"""Hand-derived known-answer scenarios for the actors: P2 switched between a remote agent and
the bot (P2_BOT / FootsiesEnv.set_opponent) and the bot playing P1 (by_example).

Expected values are derived here from the cited C#, with a separate Python restatement of
UnityEngine.Random (Xorshift128, InitState) and of BattleAI's plan choice at distance 4,
independent of the oracle and of the kernel.  A *backend* is built by ``make(p1_mode,
p2_mode, seed)`` and has ``step(p1[1] | None, p2[1] | None)``, ``state()`` (fs_arena_state
records), ``set_p2_mode(mode)`` and ``reset_hard()``.

Citations: AI = Assets/Script/BattleAI.cs, BC = Assets/Script/BattleCore.cs,
TM = Assets/Script/TrainingManager.cs, GM = Assets/Script/GameManager.cs.
"""
import numpy as np

from footsies_gym_amd import _abi

M32 = 0xFFFFFFFF
L, R, A = 1, 2, 4
MP_NEUTRAL, MP_FAR1, MP_FAR2, MP_MID1, MP_MID2 = 0, 1, 2, 3, 4
AP_NONE, AP_ONE_HIT, AP_TWO_HIT, AP_IMMEDIATE_SPECIAL, AP_DELAY_SPECIAL = 0, 1, 2, 3, 4


class Xorshift128:
    """UnityEngine.Random: InitState seeds x = seed, then y, z, w = 1812433253 * prev + 1;
    next() is Marsaglia's xorshift128 (published algorithm, restated independently)."""

    def __init__(self, seed):
        s = [seed & M32]
        for _ in range(3):
            s.append((1812433253 * s[-1] + 1) & M32)
        self.s = s

    def next(self):
        x, y, z, w = self.s
        t = (x ^ (x << 11)) & M32
        w2 = (w ^ (w >> 19) ^ t ^ (t >> 8)) & M32
        self.s = [y, z, w, w2]
        return w2

    def range(self, n):  # Random.Range(0, n) = next % n
        return self.next() % n


def move_plan_at_4(r):
    """SelectMovement for 3 < distanceX <= 4 (AI:80-98): Random.Range(0, 7)."""
    return MP_MID1 if r <= 1 else MP_MID2 if r <= 3 else MP_FAR1 if r == 4 else MP_FAR2 if r == 5 else MP_NEUTRAL


def attack_plan_at_4(r):
    """SelectAttack for 3 < distanceX <= 4 against a standing opponent (AI:146-162): Range(0, 5)."""
    return AP_NONE if r <= 1 else AP_ONE_HIT if r <= 3 else AP_DELAY_SPECIAL


def first_move_input(plan, forward):
    """The first input a movement plan enqueues (AI:192-253): forward for FAR1 / FAR2 / MID1 /
    MID2 (walks and forward dashes), 0 for NEUTRAL."""
    return 0 if plan == MP_NEUTRAL else forward


def first_attack_input(plan):
    """The first input an attack plan enqueues (AI:255-312)."""
    return 0 if plan == AP_NONE else A


def kat_switched_in_bot(make, seed=1234):
    """A game launched with a remote P2 (the FootsiesEnv `opponent` setup, GM:193-196) switches P2
    to the bot (P2_BOT, BC:158-167).  That bot was never Reset -- GameManager.botP2 is null, so
    BattleCore's Intro never reaches its Reset (BC:276-277) -- so its fightStates are null: its
    first getNextAIInput answers 0 without touching the queues or the RNG (AI:41-47), the second
    chooses plans from the FightState the first stored (distance 4.0, P1 standing: two draws),
    the third dequeues their first inputs.  A later RESET does not Reset it either: the queues
    go on where they were."""
    b = make(_abi.FS_P1_EXTERNAL, _abi.FS_P2_EXTERNAL, seed)
    rng = Xorshift128(seed)
    b.step([0], [0])                       # remote P2 plays a frame; the RNG is untouched
    assert list(b.state()[0]["rng"]) == rng.s
    b.set_p2_mode(_abi.FS_P2_BOT)
    b.step([0], [7])                       # P2 = the bot's stored input (0); the remote's 7 is ignored
    s = b.state()[0]
    assert s["p2_bot"] == 1 and s["bot_ready"][1] == 1 and s["bot_input"][1] == 0
    assert s["move_plan"] == -1 and s["attack_plan"] == -1 and list(s["rng"]) == rng.s
    assert s["prev_distance"] == np.float32(4.0) and s["prev_opponent_action"] == 0
    b.step([0], [7])                       # second call: plans chosen from (4.0, STAND)
    mp, ap = move_plan_at_4(rng.range(7)), attack_plan_at_4(rng.range(5))
    s = b.state()[0]
    assert (s["move_plan"], s["move_index"], s["attack_plan"], s["attack_index"]) == (mp, 0, ap, 0)
    assert list(s["rng"]) == rng.s and s["bot_input"][1] == 0
    assert s["actor_input"][1] == 0        # the remote actor keeps its last received action
    b.step([0], [7])                       # third call: the first inputs (P2's forward is Left)
    s = b.state()[0]
    assert s["bot_input"][1] == first_move_input(mp, L) | first_attack_input(ap)
    assert (s["move_index"], s["attack_index"]) == (1, 1) and list(s["rng"]) == rng.s
    b.reset_hard()                         # RESET: Intro does not Reset this bot; Fight's request dequeues
    s = b.state()[0]
    assert (s["move_plan"], s["move_index"], s["attack_plan"], s["attack_index"]) == (mp, 2, ap, 2)
    assert list(s["rng"]) == rng.s
    b.set_p2_mode(_abi.FS_P2_EXTERNAL)     # back to the remote actor: its action lands again
    b.step([0], [L])
    assert b.state()[0]["actor_input"][1] == L and b.state()[0]["move_index"] == 2


def kat_by_example(make, seed=99):
    """by_example (FE:230-232): --p1-bot --p1-spectator with the P2 bot (--p2-bot).  At game start
    Intro Resets P2's bot (actorP2 is botP2, BC:276-277) but not P1's (the spectator wrapper is
    no TrainingBattleAIActor, BC:274-275).  Fight's first Step (TM:59-77) asks P1's bot first: not
    ready, 0, no draw; then P2's: two draws.  The next frame P1's bot draws its plans (RNG draws
    3 and 4, before P2's dequeues), and the frame after it presses its plan's first input with
    its own forward, Right (AI:380-383)."""
    b = make(_abi.FS_P1_BOT, _abi.FS_P2_BOT, seed)
    rng = Xorshift128(seed)
    mp2, ap2 = move_plan_at_4(rng.range(7)), attack_plan_at_4(rng.range(5))
    s = b.state()[0]
    assert (s["move_plan"], s["attack_plan"], s["p1_move_plan"], s["p1_attack_plan"]) == (mp2, ap2, -1, -1)
    assert tuple(s["bot_ready"]) == (1, 1) and tuple(s["bot_input"]) == (0, 0) and list(s["rng"]) == rng.s
    assert s["p1_prev_distance"] == np.float32(4.0) and s["p1_prev_opponent_action"] == 0
    b.step(None, None)                     # both inputs 0; P1's bot chooses, P2's dequeues
    mp1, ap1 = move_plan_at_4(rng.range(7)), attack_plan_at_4(rng.range(5))
    s = b.state()[0]
    assert (s["p1_move_plan"], s["p1_move_index"], s["p1_attack_plan"], s["p1_attack_index"]) == (mp1, 0, ap1, 0)
    assert s["bot_input"][0] == 0 and s["bot_input"][1] == first_move_input(mp2, L) | first_attack_input(ap2)
    assert list(s["rng"]) == rng.s
    b.step(None, None)
    s = b.state()[0]
    assert s["bot_input"][0] == first_move_input(mp1, R) | first_attack_input(ap1)
    assert s["actor_input"][0] == 0        # no remote P1: nothing was ever received


ALL = {"switched_in_bot": kat_switched_in_bot, "by_example": kat_by_example}


class OracleActors:
    """kat_actors backend over the CPU oracle (test infrastructure)."""

    def __init__(self, oracle_lib, p1_mode, p2_mode, seed):
        self.o = oracle_lib.Oracle(1, p2_mode=p2_mode, p1_mode=p1_mode, base_seed=seed)

    def step(self, p1, p2):
        self.o.step(None if p1 is None else np.array(p1, np.uint8), None if p2 is None else np.array(p2, np.uint8))

    def state(self):
        return self.o.state()

    def set_p2_mode(self, mode):
        assert self.o.set_p2_mode(mode) == 0

    def reset_hard(self):
        self.o.reset(flags=_abi.FS_RESET_HARD)


class SimActors:
    """kat_actors backend over the HIP path (FootsiesSim, one arena)."""
    P1 = {_abi.FS_P1_EXTERNAL: "external", _abi.FS_P1_BOT: "bot"}
    P2 = {_abi.FS_P2_EXTERNAL: "external", _abi.FS_P2_BOT: "bot", _abi.FS_P2_NOOP: "noop"}

    def __init__(self, p1_mode, p2_mode, seed):
        from footsies_gym_amd.simulator import FootsiesSim
        self.sim = FootsiesSim(1, p2_mode=self.P2[p2_mode], p1_mode=self.P1[p1_mode], seed=seed)

    def step(self, p1, p2):
        self.sim.step(None if p1 is None else np.array(p1, np.uint8),
                      None if p2 is None or self.sim.p2_mode != "external" else np.array(p2, np.uint8))

    def state(self):
        return self.sim.get_state()

    def set_p2_mode(self, mode):
        self.sim.set_p2_mode(self.P2[mode])

    def reset_hard(self):
        self.sim.reset(hard=True)
