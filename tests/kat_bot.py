"""Hand-derived known answers for the scripted bot's plan logic (VERDICT r02 missing #1).

Everything expected here is restated directly from the C# (AI = Assets/Script/BattleAI.cs),
independently of the oracle's and the kernel's bot tables:

* SelectMovement / SelectAttack (AI:68-190) as the explicit if / else chains they are, every
  distance bucket with its own Random.Range size and outcome map;
* the isOpponentDamage / GuardBreak / SpecialAttack -> TwoHit rule that draws nothing (AI:130-135),
  the 3 < d <= 4 NormalAttack -> TwoHit rule that draws nothing (AI:146-150), and NoAttack at
  d > 4 still drawing (AI:136-143);
* the queue contents of every plan, built by transliterating AddFarApproach1 .. AddDelaySpecial-
  Attack and their helpers (AI:192-342) -- including AddBackwardDashInputQueue, which enqueues
  FORWARD, 0, FORWARD (AI:337-342) -- with P2's forward = Left and P1's = Right (AI:380-388);
* getNextAIInput's order (AI:41-66): the movement queue is dequeued or, when empty, refilled by a
  draw; then the attack queue likewise; a refill returns no input from that queue this call;
* UpdateFightState's ascending copy loop (AI:358-361): fightStates[5] is the PREVIOUS call's
  state, so the decision reads the loaded (prev_distance, prev_opponent_action), never the
  current positions, and the call stores the current ones for the next call.

UnityEngine.Random is Xorshift128 with Range(0, n) = next % n (tests/kat_actors.py, itself an
independent restatement; the engine's own implementation stays unpinned).

Each case is one arena loaded through the canonical state (fs_arena_state): both fighters
standing at the game's start positions (x = -2 / +2, which neither push nor move with no input),
P2's bot ready with input 0, the bot's queues and FightState and the RNG set per case; one step
with no P1 input; then the bot's fields are read back.  The movement / attack plan ids are the
canonical state's enumeration (include/footsies.h: MP_* / AP_* order of fs_internal.h).
"""
import numpy as np

from footsies_gym_amd import _abi
from tests.kat_actors import Xorshift128

L, R, A = 1, 2, 4
# canonical plan ids (fs_arena_state.move_plan / attack_plan)
MP_NEUTRAL, MP_FAR1, MP_FAR2, MP_MID1, MP_MID2, MP_FALLBACK1, MP_FALLBACK2 = range(7)
AP_NONE, AP_ONE_HIT, AP_TWO_HIT, AP_IMMEDIATE_SPECIAL, AP_DELAY_SPECIAL = range(5)
STAND, N_ATTACK, B_ATTACK, N_SPECIAL, B_SPECIAL = 0, 100, 105, 110, 115
DAMAGE, GUARD_M, GUARD_STAND, GUARD_CROUCH, GUARD_BREAK = 200, 301, 305, 306, 310


# -- the plans (AI:192-342), one transliterated builder per C# method --------------------------
def _move_plan(plan, fwd, back):
    q = []

    def forward(n):  # AddForwardInputQueue (AI:314-320)
        q.extend([fwd] * n)

    def backward(n):  # AddBackwardInputQueue (AI:322-328)
        q.extend([back] * n)

    def forward_dash():  # AddForwardDashInputQueue (AI:330-335)
        q.extend([fwd, 0, fwd])

    def backward_dash():  # AddBackwardDashInputQueue (AI:337-342): forward inputs, as written
        q.extend([fwd, 0, fwd])

    if plan == MP_NEUTRAL:  # AddNeutralMovement (AI:192-200)
        q.extend([0] * 30)
    elif plan == MP_FAR1:  # AI:202-210
        forward(40)
        backward(10)
        forward(30)
        backward(10)
    elif plan == MP_FAR2:  # AI:212-220
        forward_dash()
        backward(25)
        forward_dash()
        backward(25)
    elif plan == MP_MID1:  # AI:222-230
        forward(30)
        backward(10)
        forward(20)
        backward(10)
    elif plan == MP_MID2:  # AI:232-238
        forward_dash()
        backward(30)
    elif plan == MP_FALLBACK1:  # AI:240-245
        backward(60)
    elif plan == MP_FALLBACK2:  # AI:247-253
        backward_dash()
        backward(60)
    return q


def _attack_plan(plan):
    if plan == AP_NONE:  # AddNoAttack (AI:255-263)
        return [0] * 30
    if plan == AP_ONE_HIT:  # AI:265-274
        return [A] + [0] * 18
    if plan == AP_TWO_HIT:  # AI:276-290
        return [A] + [0] * 3 + [A] + [0] * 18
    if plan == AP_IMMEDIATE_SPECIAL:  # AI:292-301
        return [A] * 60 + [0]
    if plan == AP_DELAY_SPECIAL:  # AI:303-312
        return [A] * 120 + [0]
    raise ValueError(plan)


def move_plan(plan, player1=False):
    """The queued inputs of a movement plan for P2's bot (forward = Left) or P1's (Right)."""
    return _move_plan(plan, R, L) if player1 else _move_plan(plan, L, R)


def attack_plan(plan):
    return _attack_plan(plan)


# -- the choices (AI:68-190) ----------------------------------------------------------------------
def select_movement(d, rng):
    """SelectMovement (AI:68-126): the plan, drawing from rng."""
    if d > 4.0:
        return MP_FAR1 if rng.range(2) == 0 else MP_FAR2
    if d > 3.0:
        r = rng.range(7)
        return MP_MID1 if r <= 1 else MP_MID2 if r <= 3 else MP_FAR1 if r == 4 else MP_FAR2 if r == 5 \
            else MP_NEUTRAL
    if d > 2.5:
        r = rng.range(5)
        return [MP_MID1, MP_MID2, MP_FALLBACK1, MP_FALLBACK2, MP_NEUTRAL][r]
    if d > 2.0:
        r = rng.range(4)
        return MP_FALLBACK1 if r == 0 else MP_FALLBACK2 if r == 1 else MP_NEUTRAL
    r = rng.range(3)
    return MP_FALLBACK1 if r == 0 else MP_FALLBACK2 if r == 1 else MP_NEUTRAL


def select_attack(d, opp, rng):
    """SelectAttack (AI:128-190) against an opponent whose raw actionID was `opp`."""
    if opp in (DAMAGE, GUARD_BREAK, N_SPECIAL, B_SPECIAL):  # AI:130-135, no draw
        return AP_TWO_HIT
    if d > 4.0:  # AI:136-143: NoAttack is drawn too
        return AP_NONE if rng.range(4) <= 3 else AP_DELAY_SPECIAL
    if d > 3.0:
        if opp in (N_ATTACK, B_ATTACK):  # AI:146-150, no draw
            return AP_TWO_HIT
        r = rng.range(5)
        return AP_NONE if r <= 1 else AP_ONE_HIT if r <= 3 else AP_DELAY_SPECIAL
    if d > 2.5:
        r = rng.range(3)
        return [AP_NONE, AP_ONE_HIT, AP_TWO_HIT][r]
    if d > 2.0:
        r = rng.range(6)
        return AP_ONE_HIT if r <= 1 else AP_TWO_HIT if r <= 3 else AP_IMMEDIATE_SPECIAL if r == 4 \
            else AP_DELAY_SPECIAL
    return AP_ONE_HIT if rng.range(3) == 0 else AP_TWO_HIT


def next_input(q_move, q_attack, prev_d, prev_opp, rng, player1=False):
    """One getNextAIInput (AI:41-66) from (plan, dequeued) queues (plan -1 = empty) and the
    previous call's FightState; returns (input, new move queue, new attack queue)."""
    inp = 0
    mp, mi = q_move
    if mp >= 0:
        seq = move_plan(mp, player1)
        inp |= seq[mi]
        q_move = (mp, mi + 1) if mi + 1 < len(seq) else (-1, 0)
    else:
        q_move = (select_movement(prev_d, rng), 0)
    ap, ai = q_attack
    if ap >= 0:
        seq = attack_plan(ap)
        inp |= seq[ai]
        q_attack = (ap, ai + 1) if ai + 1 < len(seq) else (-1, 0)
    else:
        q_attack = (select_attack(prev_d, prev_opp, rng), 0)
    return inp, q_move, q_attack


# -- the cases ------------------------------------------------------------------------------------
# distances: one inside each bucket and each bucket edge with its float32 neighbours
_F = np.float32
_EDGES = [_F(4.0), _F(3.0), _F(2.5), _F(2.0)]
DISTANCES = [_F(6.5), _F(3.5), _F(2.75), _F(2.25), _F(1.0), _F(0.0)] + \
    [e for x in _EDGES for e in (x, np.nextafter(x, _F(9)), np.nextafter(x, _F(-9)))]
OPPONENTS = [STAND, N_ATTACK, B_ATTACK, N_SPECIAL, B_SPECIAL, DAMAGE, GUARD_M, GUARD_STAND, GUARD_CROUCH,
             GUARD_BREAK]


def build_cases(seed=0x5EED):
    """(name, prev_distance, prev_opponent, rng state, move queue, attack queue, player1) tuples:
    - every distance x every opponent with both queues empty, several RNG states each (draw sizes,
      outcome maps, forced TwoHit, d > 4 NoAttack drawing, the previous-state rule);
    - one queue busy, the other empty (one draw only, from the right bucket);
    - every index of every plan, both queues busy (the plan contents; no draws)."""
    rs = np.random.default_rng(seed)
    cases = []
    for d in DISTANCES:
        for o in OPPONENTS:
            for k in range(6):
                cases.append(("select d=%r opp=%d #%d" % (float(d), o, k), d, o,
                              [int(x) for x in rs.integers(1, 2**32, 4)], (-1, 0), (-1, 0), False))
    for d in DISTANCES:
        for k in range(4):
            rng = [int(x) for x in rs.integers(1, 2**32, 4)]
            cases.append(("move busy d=%r #%d" % (float(d), k), d, STAND, rng, (MP_MID1, 5), (-1, 0), False))
            cases.append(("attack busy d=%r #%d" % (float(d), k), d, STAND, rng, (-1, 0), (AP_NONE, 7), False))
    for p1 in (False, True):
        for mp in range(7):
            for i in range(len(move_plan(mp))):
                cases.append(("move plan %d[%d] p1=%d" % (mp, i, p1), _F(3.5), STAND,
                              [int(x) for x in rs.integers(1, 2**32, 4)], (mp, i), (AP_DELAY_SPECIAL, i % 120), p1))
        for ap in range(5):
            for i in range(len(attack_plan(ap))):
                cases.append(("attack plan %d[%d] p1=%d" % (ap, i, p1), _F(3.5), STAND,
                              [int(x) for x in rs.integers(1, 2**32, 4)], (MP_FAR1, i % 90), (ap, i), p1))
    return cases


def load_cases(base, cases, player1):
    """Arena states (copies of `base[0]`, a fresh handle's state) carrying the cases."""
    st = np.repeat(base[:1], len(cases), axis=0)
    for i, (_, d, o, rng, qm, qa, _p1) in enumerate(cases):
        s = st[i]
        for k, x in ((0, -2.0), (1, 2.0)):
            f = s["f"][k]
            f["position_x"], f["action_id"], f["action_frame"], f["hit_count"], f["hitstun"] = x, STAND, 3, 0, 0
            f["vital"], f["guard"], f["buffer_action_id"], f["reserve_action_id"] = 1, 3, -1, -1
            f["input_dir_history"], f["attack_hold"] = 0, 0
            f["is_input_backward"] = f["is_reserve_proximity_guard"] = f["has_won"] = 0
        s["frame_count"], s["recording_count"], s["reset_pending"], s["has_terminated"] = 100, 101, 0, 0
        s["rng"] = rng
        s["bot_ready"] = (1, 1)
        s["bot_input"] = (0, 0)
        if player1:  # the case is P1's bot; P2's keeps busy queues (no draws of its own)
            s["p1_move_plan"], s["p1_move_index"], s["p1_attack_plan"], s["p1_attack_index"] = qm + qa
            s["p1_prev_distance"], s["p1_prev_opponent_action"] = d, o
            s["move_plan"], s["move_index"], s["attack_plan"], s["attack_index"] = MP_FAR1, 0, AP_DELAY_SPECIAL, 0
            s["prev_distance"], s["prev_opponent_action"] = _F(3.5), STAND
        else:
            s["move_plan"], s["move_index"], s["attack_plan"], s["attack_index"] = qm + qa
            s["prev_distance"], s["prev_opponent_action"] = d, o
    return st


def check(after, cases, player1):
    """Compare one stepped batch with the restatement; returns the coverage seen."""
    seen = set()
    for i, (name, d, o, rng0, qm, qa, _p1) in enumerate(cases):
        rng = Xorshift128(0)
        rng.s = list(rng0)
        inp, nm, na = next_input(qm, qa, float(d), o, rng, player1)
        s = after[i]
        pre = "p1_" if player1 else ""
        got = (int(s[pre + "move_plan"]), int(s[pre + "move_index"]), int(s[pre + "attack_plan"]),
               int(s[pre + "attack_index"]))
        assert got == nm + na, "%s: queues %s, expected %s" % (name, got, nm + na)
        assert int(s["bot_input"][0 if player1 else 1]) == inp, "%s: input %d, expected %d" % (
            name, int(s["bot_input"][0 if player1 else 1]), inp)
        assert [int(x) for x in s["rng"]] == rng.s, "%s: RNG %s, expected %s" % (name, list(s["rng"]), rng.s)
        # the call stored the CURRENT FightState for the next call (fighters at -2 / +2, P1 standing)
        assert s[pre + "prev_distance"] == _F(4.0) and int(s[pre + "prev_opponent_action"]) == STAND, name
        draws = sum(1 for a, b in zip(rng0, rng.s) if a != b) > 0
        seen.add((name.split()[0], qm[0] < 0 and nm[0], qa[0] < 0 and na[0], draws))
    return seen


def run(make):
    """make(n, player1) -> backend with get_state() / set_state(st) / step() (no P1 input)."""
    cases = build_cases()
    for player1 in (False, True):
        mine = [c for c in cases if c[6] == player1]
        b = make(len(mine), player1)
        b.set_state(load_cases(b.get_state(), mine, player1))
        b.step()
        check(b.get_state(), mine, player1)
    return cases


def coverage(cases):
    """Which outcomes the P2 selection cases reach, per bucket (a property of the cases and the
    restatement, checked so the sampled RNG states provably cover every branch)."""
    out = {}
    for (name, d, o, rng0, qm, qa, p1) in cases:
        if p1 or not name.startswith("select"):
            continue
        rng = Xorshift128(0)
        rng.s = list(rng0)
        _, nm, na = next_input(qm, qa, float(d), o, rng, False)
        out.setdefault(("move", bucket(d)), set()).add(nm[0])
        out.setdefault(("attack", bucket(d), o in (DAMAGE, GUARD_BREAK, N_SPECIAL, B_SPECIAL),
                        o in (N_ATTACK, B_ATTACK)), set()).add(na[0])
    return out


def bucket(d):
    d = float(d)
    return 0 if d > 4 else 1 if d > 3 else 2 if d > 2.5 else 3 if d > 2 else 4


class OracleBot:
    """run() backend over the CPU oracle (test infrastructure)."""

    def __init__(self, oracle_lib, n, player1):
        self.o = oracle_lib.Oracle(n, p2_mode=_abi.FS_P2_BOT,
                                   p1_mode=_abi.FS_P1_BOT if player1 else _abi.FS_P1_EXTERNAL)
        self.n, self.player1 = n, player1

    def get_state(self):
        return self.o.state()

    def set_state(self, st):
        assert self.o.set_state(st) == 0

    def step(self):
        self.o.step(None if self.player1 else np.zeros(self.n, np.uint8))


class SimBot:
    """run() backend over the HIP path."""

    def __init__(self, n, player1):
        from footsies_gym_amd.simulator import FootsiesSim
        self.sim = FootsiesSim(n, p2_mode="bot", p1_mode="bot" if player1 else "external", seed=0)
        self.n, self.player1 = n, player1

    def get_state(self):
        return self.sim.get_state()

    def set_state(self, st):
        self.sim.set_state(st)

    def step(self):
        self.sim.step(None if self.player1 else np.zeros(self.n, np.uint8))
