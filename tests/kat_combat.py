"""Hand-derived known-answer scenarios for combat: landed attacks, hitstun, cancels, KOs,
trades, invulnerable frames, the WIN loop and hitstun carried through the auto-reset burst.

Like tests/kat_scenarios.py, every expected value is derived here from data/f00.json (the
reference's F00 assets, re-extracted byte-identically by tests/test_tables.py) and the cited
C#, with plain numpy float32 arithmetic in the C# operand order -- independent of the oracle
and of the kernel.  A *backend* has ``reset()``, ``step(p1[1], p2[1]) -> outputs``,
``env_state()``, and for the scenarios that start from a loaded position ``state()`` /
``set_state(records)``.  Scenarios run with dense rewards and same-step auto-reset.

Citations: BC = Assets/Script/BattleCore.cs, F = Assets/Script/Fighter.cs,
FE = footsies-gym/footsies_gym/envs/footsies.py, ACT = Assets/Fighter/F00/Actions/*.asset,
ATK = Assets/Fighter/F00/F00_AttackDataContainer.asset.
"""
import json
import os

import numpy as np

F32 = np.float32
DT = F32(0.02)
L, R, A = 1, 2, 4
STAND, FORWARD, DASH_B = 0, 1, 11
N_ATTACK, N_SPECIAL, B_SPECIAL, DAMAGE, DEAD, WIN = 100, 110, 115, 200, 500, 510

_DATA = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "f00.json")))
ACTIONS = {a["id"]: a for a in _DATA["actions"]}
ATTACKS = {a["id"]: a for a in _DATA["attacks"]}


def velocity(action, frame):
    """ActionData.GetMovementData (AD:150-168): the first movement window holding the frame."""
    for m in ACTIONS[action]["movements"]:
        if m["win"][0] <= frame <= m["win"][1]:
            return m["velocity_x"]
    return 0.0


def step_x(x, speed_or_v, sign, walk=None):
    """One frame of UpdateMovement (F:291-319) in float32: FORWARD `x += speed * sign * dt`,
    BACKWARD `x -= speed * sign * dt`, otherwise `x += v * sign * dt` for v != 0."""
    t = F32(F32(F32(speed_or_v) * F32(sign)) * DT)
    if walk == "backward":
        return F32(x - t)
    if speed_or_v == 0:
        return x
    return F32(x + t)


def run(backend, p1, p2, steps, start=0):
    """Drive one arena from its current state for `steps` ticks; returns per-tick env states
    and outputs keyed by tick."""
    st, out = {}, {}
    for t in range(start, start + steps):
        o = backend.step(np.array([p1(t)], np.uint8), np.array([p2(t)], np.uint8))
        st[t] = backend.env_state()[0].copy()
        out[t] = {k: np.array(v, copy=True) for k, v in o.items()}
    return st, out


def approach(n):
    """Both fighters walk forward for n frames from the start positions (-2, 2): P1 holds Right,
    P2 holds Left (both their forward, F:642-653); FORWARD moves 2.2 units/s (F00.asset)."""
    x1, x2 = F32(-2), F32(2)
    for _ in range(n):
        x1, x2 = step_x(x1, 2.2, 1), step_x(x2, 2.2, -1)
    return x1, x2


def kat_landed_n_attack(backend):
    """After 17 frames of walking in (distance ~2.504), P1 jabs a standing P2.  N_ATTACK's real
    hitbox (ACT/N_ATTACK.asset: frames 4-5, rect x 0.9 w 1.8 -> [x1, x1 + 1.8]) reaches P2's
    base hurtbox ([x2 - 0.75, x2 + 0.75], F00.asset) on frame 4.  NotifyDamaged (F:357-398):
    guard damage 1 applies even unguarded (3 -> 2), P2 is not blocking, vital damage 0, DAMAGE
    is set; both fighters get hitStun 12 (ATK N_ATTACK, BC:576-578).  Dense reward +0.3 for
    P2's guard drop (FE:393-394).  For 12 ticks both action frames freeze while the stun counts
    down and nobody moves (F:149-154, 293-294); the tick the stun reaches 0 still freezes the
    frame but P2 moves with DAMAGE frame 0's velocity -3 (knocked back, away from P1)."""
    backend.reset()
    x1, x2 = approach(17)
    assert x2 - x1 <= F32(2.55) and x2 - x1 > F32(1.4)
    st, out = run(backend, lambda t: R if t < 17 else (A if t == 17 else 0), lambda t: L if t < 17 else 0, 40)
    assert (st[16]["p1Position"], st[16]["p2Position"]) == (x1, x2)
    for t in range(17, 21):
        assert st[t]["p1Move"] == N_ATTACK and st[t]["p1MoveFrame"] == t - 17 and st[t]["p2Move"] == STAND, t
        assert st[t]["p2Guard"] == 3 and out[t]["reward"][0] == 0.0
    h = st[21]
    assert (h["p1Move"], h["p1MoveFrame"], h["p2Move"], h["p2MoveFrame"]) == (N_ATTACK, 4, DAMAGE, 0)
    assert (h["p1Hitstun"], h["p2Hitstun"], h["p1Guard"], h["p2Guard"], h["p2Vital"]) == (12, 12, 3, 2, 1)
    assert out[21]["reward"][0] == 0.3 and not out[21]["terminated"][0]
    for k in range(1, 12):
        s = st[21 + k]
        assert (s["p1Hitstun"], s["p2Hitstun"]) == (12 - k, 12 - k), k
        assert (s["p1MoveFrame"], s["p2MoveFrame"]) == (4, 0) and (s["p1Position"], s["p2Position"]) == (x1, x2), k
    s = st[33]
    assert (s["p1Hitstun"], s["p2Hitstun"], s["p1MoveFrame"], s["p2MoveFrame"]) == (0, 0, 4, 0)
    assert s["p1Position"] == x1 and s["p2Position"] == step_x(x2, velocity(DAMAGE, 0), -1)
    assert (st[34]["p1MoveFrame"], st[34]["p2MoveFrame"]) == (5, 1)


def kat_cancel_needs_a_hit(backend, land):
    """N_ATTACK -> N_SPECIAL cancel (F:241-246, 472-510; ACT/N_ATTACK.asset cancels: frames 1-3
    buffer N_SPECIAL, 4-5 execute): a second Attack press on frame 2 leaves N_SPECIAL in
    bufferActionID.  UpdateActionRequest takes a buffered action only when canCancelAttack()
    -- canCancelOnWhiff is false, so only after the attack hit (F:222-229, 531-539) -- and not
    in hitstun.  Landed (distance ~2.504): the hit on frame 4 stuns 12; on the tick the stun
    reaches 0 the buffer is taken: N_SPECIAL frame 0, 12 ticks after the hit.  Whiffed (no
    approach, distance 4): the buffer is never taken, N_ATTACK runs its 22 frames."""
    backend.reset()
    n = 17 if land else 0
    press = {n, n + 2}
    st, _ = run(backend, lambda t: R if t < n else (A if t in press else 0), lambda t: L if t < n else 0, n + 30)
    if land:
        assert st[n + 4]["p2Move"] == DAMAGE and st[n + 4]["p1Hitstun"] == 12
        for t in range(n + 4, n + 16):
            assert st[t]["p1Move"] == N_ATTACK and st[t]["p1MoveFrame"] == 4, t
        assert st[n + 16]["p1Move"] == N_SPECIAL and st[n + 16]["p1MoveFrame"] == 0 and st[n + 16]["p1Hitstun"] == 0
    else:
        for t in range(n, n + 22):
            assert st[t]["p1Move"] == N_ATTACK and st[t]["p1MoveFrame"] == t - n, t
        assert st[n + 22]["p1Move"] == STAND and st[n + 4]["p2Guard"] == 3


def charge_then(hold, x1=F32(-2)):
    """P1 x at each N_SPECIAL frame f after a charge released at tick `hold` (CheckSpecialAttack
    Input, F:569-583): the move starts at frame 0 on the release tick and moves with its own
    velocities (ACT/N_SPECIAL.asset) from that tick on."""
    xs = {}
    for f in range(44):
        x1 = step_x(x1, velocity(N_SPECIAL, f), 1)
        xs[hold + f] = x1
    return xs


def kat_special_ko_reward(backend):
    """A dense-reward episode ending in a KO.  P2 walks in 34 frames (distance ~2.504) and
    stands; P1 lands an N_ATTACK (guard 3 -> 2: +0.3).  Once that is over P1 charges Attack 59
    frames and releases: N_SPECIAL (ATK: vital damage 1, guard damage 1, hitStun 0) lands on
    frame 11 on the knocked-back P2 -- guard 2 -> 1 (+0.3) and vital 1 -> 0, DEAD (F:388-395).
    The battle is over (BC:212-213): terminated, reward = 0.3 + (1 - cumulative 0.6)
    (FE:388-405, in FE's float64 order), so the episode's rewards sum to 1.  The terminal
    observation shows DEAD as STAND (FE:537-549).  P1 is the sole survivor, so the End tick makes
    it win (BC:310-323, F:461-464): its UpdateActionRequest returns at the WIN request
    (F:204-208) and keeps isInputBackward -- P1 held Left on the KO tick -- through the reset,
    while the loser's is cleared (its input was cleared at KO, BC:296-299).  The same step
    returns state(-1) (same-step auto-reset)."""
    backend.reset()
    jab, hold_from = 34, 70
    rel = hold_from + 59
    ko = rel + 11

    def p1(t):
        if t == jab or hold_from <= t < rel:
            return A
        return L if t == ko else 0
    st, out = run(backend, p1, lambda t: L if t < jab else 0, ko + 1)
    x2 = F32(2)
    for _ in range(jab):
        x2 = step_x(x2, 2.2, -1)
    assert x2 - F32(-2) <= F32(2.55)
    hit = jab + 4
    assert st[hit]["p2Move"] == DAMAGE and st[hit]["p2Guard"] == 2 and out[hit]["reward"][0] == 0.3
    # DAMAGE knocks P2 back once its stun is over (velocities by frame, ACT/DAMAGE.asset)
    for t in range(hit + 1, ko):  # (the KO tick itself reports the next episode's state(-1))
        if st[t]["p2Move"] == DAMAGE and st[t]["p2Hitstun"] == 0:
            x2 = step_x(x2, velocity(DAMAGE, st[t]["p2MoveFrame"]), -1)
        assert st[t]["p2Position"] == x2, t
    xs = charge_then(rel)
    assert st[rel]["p1Move"] == N_SPECIAL and st[rel]["p1MoveFrame"] == 0
    assert st[ko - 1]["p2Vital"] == 1 and st[ko - 1]["p1Position"] == xs[ko - 1]
    assert x2 - F32(0.75) <= xs[ko] + F32(2.0)  # N_SPECIAL's hitbox [x1, x1 + 2] reaches P2
    o = out[ko]
    assert o["terminated"][0] == 1 and o["truncated"][0] == 0
    assert o["reward"][0] == 0.3 + (1 - (0.3 + 0.3))
    assert abs(sum(float(out[t]["reward"][0]) for t in out) - 1.0) < 1e-12
    assert o["final_move"][0, 1] == 0 and o["final_move_frame"][0, 1] == 0.0  # DEAD -> STAND
    assert o["final_guard"][0, 1] == 1
    s = backend.env_state()[0]
    assert s["globalFrame"] == -1 and (s["p1Vital"], s["p2Vital"], s["p1Guard"], s["p2Guard"]) == (1, 1, 3, 3)
    cs = backend.state()[0]
    assert cs["f"][0]["is_input_backward"] == 1 and cs["f"][1]["is_input_backward"] == 0
    assert cs["f"][0]["has_won"] == 0  # SetupBattleStart clears hasWon (F:128)


def kat_trade_carries_hitstun(backend):
    """A same-tick trade and hitstun carried through the auto-reset burst.  Both fighters start
    still; P1 charges Attack 59 frames (N_SPECIAL from tick 59) while P2 walks in 12 frames and
    jabs at tick 66, so on tick 70 P1's N_SPECIAL (frame 11) and P2's N_ATTACK (frame 4) are
    both active.  UpdateHitboxHurtboxCollision (BC:521-591) resolves P1 first: P2 dies (DEAD,
    hit count reset, hitStun 0 on both).  Then P2 attacks with the boxes UpdateBoxes built
    before the hit: its stale N_ATTACK hitbox still hits P1 (DAMAGE, guard 3 -> 2, hitStun 12 on
    both).  P1 survives (vital damage 0) and wins.  Reward: guard drops on both sides cancel,
    +1 for the KO.  SetupBattleStart does not reset currentHitStunFrame (F:120-135), so the stun
    survives the burst, minus the End tick's and the Intro tick's decrements (BC:329-345,
    371-381): state(-1) shows hitstun 10 for both and action frame 0 (frozen in the Intro tick)."""
    backend.reset()
    rel, walk, jab = 59, 12, 66
    st, out = run(backend, lambda t: A if t < rel else 0, lambda t: L if t < walk else (A if t == jab else 0), 71)
    x2 = F32(2)
    for _ in range(walk):
        x2 = step_x(x2, 2.2, -1)
    xs = charge_then(rel)
    d = x2 - xs[70]
    assert d <= F32(2.55) and d > F32(1.4)  # both reach; the pushboxes stay apart
    for t in range(rel, 70):
        assert st[t]["p2Vital"] == 1 and st[t]["p1Vital"] == 1 and st[t]["p1Move"] == N_SPECIAL, t
    assert st[69]["p2Move"] == N_ATTACK and st[69]["p2MoveFrame"] == 3
    o = out[70]
    assert o["terminated"][0] == 1 and o["reward"][0] == 1.0
    assert tuple(o["final_move"][0]) == (9, 0)  # P1 DAMAGE (index 9), P2 DEAD -> STAND
    assert tuple(o["final_hitstun"][0]) == (12, 12) and tuple(o["final_guard"][0]) == (2, 2)
    # state(-1) of the next episode, returned by the same step
    assert o["frame"][0] == -1 and tuple(o["hitstun"][0]) == (10, 10)
    assert tuple(o["move"][0]) == (0, 0) and tuple(o["move_frame"][0]) == (0.0, 0.0)
    s2, _ = run(backend, lambda t: 0, lambda t: 0, 11, start=71)
    for k in range(10):
        assert (s2[71 + k]["p1Hitstun"], s2[71 + k]["p1MoveFrame"]) == (9 - k, 0), k
    assert s2[81]["p1MoveFrame"] == 1


def kat_double_ko(backend):
    """Both charge 59 frames and release on the same tick: both N_SPECIALs land on frame 11 (the
    setup is mirror-symmetric).  P1 attacks first and kills P2 (hit count reset); P2's stale
    hitbox then kills P1.  Both vitals are 0; FootsiesEnv scores the terminal step by p2Vital
    alone (FE:388-405): +1, a P1 win; the guard drops (3 -> 2 each) cancel.  No sole survivor:
    nobody gets the WIN request (BC:310-323)."""
    backend.reset()
    st, out = run(backend, lambda t: A if t < 59 else 0, lambda t: A if t < 59 else 0, 71)
    xs = charge_then(59)
    assert F32(-xs[70]) - xs[70] <= F32(2.75)
    o = out[70]
    assert o["terminated"][0] == 1 and o["reward"][0] == 1.0
    assert tuple(o["final_move"][0]) == (0, 0) and tuple(o["final_guard"][0]) == (2, 2)
    assert st[69]["p1Vital"] == 1 and st[69]["p2Vital"] == 1


# ---------------------------------------------------------------------------------------------
# scenarios from loaded positions (fs_set_state / STATE_LOAD)
# ---------------------------------------------------------------------------------------------
def _fighter(rec, x, action, frame, guard=3):
    rec["position_x"] = x
    rec["action_id"] = action
    rec["action_frame"] = frame
    rec["vital"] = 1
    rec["guard"] = guard
    rec["hit_count"] = 0
    rec["hitstun"] = 0
    rec["buffer_action_id"] = -1
    rec["reserve_action_id"] = -1


def load(backend, p1, p2):
    """STATE_LOAD of one arena in the Fight state: fighters given as (x, action, frame)."""
    s = backend.state()
    s["frame_count"] = 100
    s["recording_count"] = 100
    s["has_terminated"] = 0
    s["reset_pending"] = 0
    _fighter(s["f"][0, 0], F32(p1[0]), *p1[1:])
    _fighter(s["f"][0, 1], F32(p2[0]), *p2[1:])
    backend.set_state(s)


def kat_invulnerable_startups(backend):
    """B_SPECIAL has no hurtbox on frames 0-5 (ACT/B_SPECIAL.asset: window 6-54) and
    DASH_BACKWARD none on frames 0-3 (window 4-21).  P2 is loaded in N_ATTACK frame 3, so its
    real hitbox ([x2 - 1.8, x2], facing left) is out on the next tick and reaches P1's hurtbox,
    when there is one; P1 is loaded in the move at frame f and ticks to f + 1.
    DASH_BACKWARD (no hitbox): frames 1-3 are not hit, frame 4 is (DAMAGE, guard 3 -> 2, stun 12,
    -0.3).  B_SPECIAL's own hitbox (frames 2-7, [x1, x1 + 1.2]) reaches P2's extended N_ATTACK
    hurtbox ([x2 - 1.6, x2], frames 4-15) and kills it (vital damage 1); P2 attacks second, with
    the hitbox built before it died (BC:521-591), so P1 is hit only if it has a hurtbox: frame 1
    nothing happens; frames 2-5 P2 dies and P1 stays in B_SPECIAL; frame 6 both are hit."""
    for f in range(4):  # DASH_BACKWARD
        backend.reset()
        load(backend, (-1.0, DASH_B, f), (1.0, N_ATTACK, 3))
        out = backend.step(np.array([0], np.uint8), np.array([0], np.uint8))
        s = backend.env_state()[0]
        hurt = f + 1 >= 4
        assert s["p2MoveFrame"] == 4 and s["p2Position"] - F32(1.8) <= s["p1Position"] + F32(0.45)
        assert (s["p1Move"] == DAMAGE) == hurt and (s["p1Guard"] == 2) == hurt, f
        assert (s["p1Hitstun"] == 12) == hurt and out["reward"][0] == (-0.3 if hurt else 0.0), f
    for f in range(6):  # B_SPECIAL
        backend.reset()
        load(backend, (-1.0, B_SPECIAL, f), (1.3, N_ATTACK, 3))
        out = backend.step(np.array([0], np.uint8), np.array([0], np.uint8))
        nf = f + 1
        if nf < 2:
            s = backend.env_state()[0]
            assert not out["terminated"][0] and (s["p1Move"], s["p1MoveFrame"], s["p1Guard"]) == (B_SPECIAL, nf, 3)
            continue
        assert out["terminated"][0] == 1 and out["reward"][0] == 1.0, f  # P2 died; +0.3 +0.7 or -0.3 +0.3 +1
        p1_hit = nf >= 6
        assert out["final_move"][0, 0] == (9 if p1_hit else 8), f  # DAMAGE / B_SPECIAL (move index)
        assert tuple(out["final_guard"][0]) == ((2, 2) if p1_hit else (3, 2)), f
        assert tuple(out["final_hitstun"][0]) == ((12, 12) if p1_hit else (0, 0)), f


def kat_win_loops_from_5(backend):
    """WIN (ACT/WIN.asset: 33 frames, isLoop, loopFromFrame 5): IncrementActionFrame past the
    last frame jumps back to 5 (F:156-165); the hasWon request of WIN on WIN changes nothing
    (F:204-208, 480-483).  Loaded in WIN at frame 31 with hasWon, the winner shows 32, then 5,
    6, ...  The observation maps WIN to STAND (FE:537-549)."""
    backend.reset()
    load(backend, (-2.0, WIN, 31), (2.0, STAND, 0))
    s = backend.state()
    s["f"][0, 0]["has_won"] = 1
    backend.set_state(s)
    frames = []
    for _ in range(4):
        out = backend.step(np.array([0], np.uint8), np.array([0], np.uint8))
        e = backend.env_state()[0]
        assert e["p1Move"] == WIN and out["move"][0, 0] == 0 and out["move_frame"][0, 0] == 0.0
        frames.append(int(e["p1MoveFrame"]))
    assert frames == [32, 5, 6, 7], frames


ALL = {
    "landed_n_attack": kat_landed_n_attack,
    "cancel_after_hit": lambda b: kat_cancel_needs_a_hit(b, True),
    "cancel_needs_hit": lambda b: kat_cancel_needs_a_hit(b, False),
    "special_ko_reward": kat_special_ko_reward,
    "trade_carries_hitstun": kat_trade_carries_hitstun,
    "double_ko": kat_double_ko,
    "invulnerable_startups": kat_invulnerable_startups,
    "win_loops_from_5": kat_win_loops_from_5,
}


class OracleKat:
    """kat_combat backend over the CPU oracle (one arena, dense reward, same-step auto-reset)."""

    def __init__(self, oracle_lib):
        from footsies_gym_amd import _abi
        self.o = oracle_lib.Oracle(1, p2_mode=_abi.FS_P2_EXTERNAL, autoreset_mode=_abi.FS_AUTORESET_SAME_STEP)

    def reset(self):
        return self.o.reset()

    def step(self, p1, p2):
        return self.o.step(p1, p2)

    def env_state(self):
        return self.o.env_state()

    def state(self):
        return self.o.state()

    def set_state(self, s):
        assert self.o.set_state(s) == 0
