"""Hand-derived known-answer scenarios for the FOOTSIES simulation.

Each scenario scripts P1/P2 inputs for one arena and states what the reference
code (cited per check) must produce.  Expected positions are computed here with
plain numpy float32 arithmetic in the C# expression order, independent of the
oracle and of the kernel.  A *backend* is any object with
``reset() -> outputs``, ``step(p1[1], p2[1]) -> outputs`` and ``env_state()``
(the Oracle binding or a FootsiesSim wrapper).

Citations: BC = Assets/Script/BattleCore.cs, F = Assets/Script/Fighter.cs,
ACT = Assets/Fighter/F00/Actions/*.asset.
"""
import numpy as np

F32 = np.float32
DT = F32(0.02)
STAND, FORWARD, BACKWARD, DASH_F, DASH_B = 0, 1, 2, 10, 11
N_ATTACK, N_SPECIAL, GUARD_M, GUARD_STAND, GUARD_CROUCH, GUARD_BREAK, GUARD_PROX = 100, 110, 301, 305, 306, 310, 350
L, R, A = 1, 2, 4


def walk(x, speed, sign, n, backward=False):
    """n frames of `position.x (+|-)= speed * sign * Time.deltaTime` (F:300, 305)."""
    xs = []
    for _ in range(n):
        t = F32(F32(F32(speed) * F32(sign)) * DT)
        x = F32(x - t) if backward else F32(x + t)
        xs.append(x)
    return xs


def move_by(x, v, sign):
    """one frame of `position.x += velocity_x * sign * Time.deltaTime` (F:316) if v != 0."""
    if v == 0:
        return x
    return F32(x + F32(F32(F32(v) * F32(sign)) * DT))


def run(backend, p1_seq, p2_seq, steps, record=None):
    """Drive one arena; returns per-step env states (fs_env_state records) and outputs."""
    backend.reset()
    states, outs = [], []
    for t in range(steps):
        a1 = p1_seq(t) if callable(p1_seq) else p1_seq[t]
        a2 = p2_seq(t) if callable(p2_seq) else p2_seq[t]
        out = backend.step(np.array([a1], np.uint8), np.array([a2], np.uint8))
        if record is None or t in record:
            states.append((t, backend.env_state()[0].copy()))
            outs.append((t, {k: np.array(v, copy=True) for k, v in out.items()}))
    return states, outs


def kat_idle(backend):
    """Nobody presses anything: STAND loops every 24 frames (ACT/STAND.asset frameCount 24:
    frame 24 ends the action and RequestAction(STAND) restarts it, F:474-478); state(-1)
    already sits at frame 1 (SetCurrentAction + one IncrementActionFrame in the Intro tick)."""
    st, _ = run(backend, lambda t: 0, lambda t: 0, 100)
    for t, s in st:
        assert s["p1Move"] == STAND and s["p2Move"] == STAND
        assert s["p1MoveFrame"] == (t + 2) % 24 and s["p2MoveFrame"] == (t + 2) % 24, t
        assert s["globalFrame"] == t
        assert s["p1Position"] == F32(-2) and s["p2Position"] == F32(2)
        assert s["p1Guard"] == 3 and s["p2Guard"] == 3 and s["p1Vital"] == 1 and s["p2Vital"] == 1


def kat_walk(backend):
    """P1 holds Right (forward, faces right) and P2 holds Right (backward, faces left) for 40
    frames: FORWARD/BACKWARD at 2.2 / 1.8 units/s (F00.asset forward/backwardMoveSpeed);
    FORWARD restarts at frame 24 (t % 24)."""
    st, _ = run(backend, lambda t: R, lambda t: R, 40)
    x1 = walk(F32(-2), 2.2, 1, 40)
    x2 = walk(F32(2), 1.8, -1, 40, backward=True)
    for t, s in st:
        assert s["p1Move"] == FORWARD and s["p2Move"] == BACKWARD, t
        assert s["p1MoveFrame"] == t % 24, t
        assert s["p1Position"] == x1[t] and s["p2Position"] == x2[t], (t, s["p1Position"], x1[t])


def kat_n_attack_whiff(backend):
    """A single Attack press from neutral starts N_ATTACK (F:241-253), 22 frames, no movement
    window; at distance 4 nothing connects; frame 22 falls back to STAND."""
    st, _ = run(backend, lambda t: A if t == 0 else 0, lambda t: 0, 30)
    for t, s in st:
        if t <= 21:
            assert s["p1Move"] == N_ATTACK and s["p1MoveFrame"] == t, t
        else:
            assert s["p1Move"] == STAND and s["p1MoveFrame"] == t - 22, t
        assert s["p2Guard"] == 3 and s["p1Position"] == F32(-2)


DASH_F_V = [5, 5, 5, 7, 7, 7, 7, 7, 7, 5, 5, 5, 2, 2, 1, 0]      # ACT/DASH_FORWARD.asset movements
DASH_B_V = [-10, -10, -10, -5, -5, -5, -5, -5, -5, -3, -3, -3, -3, -1, -1, 0]  # ACT/DASH_BACKWARD.asset


def kat_dash_forward(backend):
    """Right, neutral, Right: CheckForwardDashInput (F:585-609, dashAllowFrame 9) fires on the
    second press; DASH_FORWARD runs 16 frames with its per-frame velocities."""
    seq = [R, 0, R] + [0] * 20
    st, _ = run(backend, seq, [0] * 23, 23)
    x = walk(F32(-2), 2.2, 1, 1)[0]
    xs = {0: x, 1: x}
    for f in range(16):
        x = move_by(x, DASH_F_V[f], 1)
        xs[2 + f] = x
    for t, s in st:
        if t == 0:
            assert s["p1Move"] == FORWARD
        elif t == 1:
            assert s["p1Move"] == STAND
        elif t <= 17:
            assert s["p1Move"] == DASH_F and s["p1MoveFrame"] == t - 2, t
        else:
            assert s["p1Move"] == STAND, t
        if t <= 17:
            assert s["p1Position"] == xs[t], (t, s["p1Position"], xs[t])


def kat_dash_backward(backend):
    """Left, neutral, Left: DASH_BACKWARD (22 frames; velocities on frames 0-15 only)."""
    seq = [L, 0, L] + [0] * 25
    st, _ = run(backend, seq, [0] * 28, 28)
    x = walk(F32(-2), 1.8, 1, 1, backward=True)[0]
    xs = {0: x, 1: x}
    for f in range(22):
        x = move_by(x, DASH_B_V[f] if f < 16 else 0, 1)
        xs[2 + f] = x
    for t, s in st:
        if 2 <= t <= 23:
            assert s["p1Move"] == DASH_B and s["p1MoveFrame"] == t - 2, t
            assert s["p1Position"] == xs[t], (t, s["p1Position"], xs[t])
        elif t >= 24:
            assert s["p1Move"] == STAND, t


def kat_charge_special(backend, hold):
    """Hold Attack `hold` frames from t=0, release: CheckSpecialAttackInput (F:569-583) needs
    inputUp[0] & Attack and Attack on input[1..59], i.e. 59 held frames."""
    st, _ = run(backend, lambda t: A if t < hold else 0, lambda t: 0, hold + 2)
    s = dict(st)[hold]
    if hold >= 59:
        assert s["p1Move"] == N_SPECIAL and s["p1MoveFrame"] == 0, (hold, s["p1Move"])
    else:
        assert s["p1Move"] == STAND, (hold, s["p1Move"])
    assert dict(st)[0]["p1Move"] == N_ATTACK  # the initial press was an N_ATTACK


def kat_proximity_guard(backend, back_at_attack):
    """P2 walks forward 7 frames (x2 ~ 1.692) then presses Attack: N_ATTACK's proximity
    hitbox (ACT/N_ATTACK.asset: frames 0-5, rect x 1.5 w 3) reaches P1's hurtbox while the
    real one does not.  If P1 was pressing back on that frame (isInputBackward), the collision
    sets isReserveProximityGuard (F:400-406, BC:583-586) and the next back press requests
    GUARD_PROXIMITY instead of BACKWARD (F:273-279)."""
    def p1(t):
        if t == 7:
            return L if back_at_attack else 0
        return L if t == 8 else 0

    def p2(t):
        return L if t < 7 else (A if t == 7 else 0)
    st, _ = run(backend, p1, p2, 10)
    d = dict(st)
    x2 = walk(F32(2), 2.2, -1, 7)[-1]
    assert d[6]["p2Position"] == x2 and x2 <= F32(1.714)
    assert d[7]["p2Move"] == N_ATTACK and d[7]["p1Guard"] == 3
    assert d[8]["p1Move"] == (GUARD_PROX if back_at_attack else BACKWARD), d[8]["p1Move"]


def kat_recording_cap(backend):
    """RecordInput stops after 60*60*5 = 18000 frames (BC:67, 595-596): MostRecentAction then
    stays at the input of frame 17999."""
    rec = {17998, 17999, 18000, 18005}
    _, outs = run(backend, lambda t: R if t == 17999 else 0, lambda t: 0, 18006, record=rec)
    o = dict(outs)
    assert o[17998]["action"][0, 0] == 0
    for t in (17999, 18000, 18005):
        assert o[t]["action"][0, 0] == R, (t, o[t]["action"])
        assert o[t]["frame"][0] == t


def kat_guard_break(backend):
    """P1 holds back (BACKWARD counts as blocking, F:370-371) and walks to the wall; P2 closes in
    and jabs.  Every connecting attack deals 1 guard damage (F:360-368); guards 3 -> 2 -> 1 -> 0
    come with a guard action and a 12/15-frame stun on both fighters and a -0.3 dense reward
    (footsies.py:393-394); the fourth guard-damaging hit breaks the guard: guard stays 0, the
    guard action is set with GUARD_BREAK reserved and 30 frames of stun (F:373-379, 446-454),
    after which P1 enters GUARD_BREAK."""
    backend.reset()
    last = None
    events = []  # (t, guard_before, guard_after, p1Move, p1Hitstun, reward)
    broke_at = None
    saw_guard_break_action = False
    for t in range(600):
        s = backend.env_state()[0]
        dist = s["p2Position"] - s["p1Position"]
        a2 = L if dist > 2.2 else (A if t % 3 == 0 else 0)
        out = backend.step(np.array([L], np.uint8), np.array([a2], np.uint8))
        s2 = backend.env_state()[0]
        assert not out["terminated"][0], "P1 must never take vital damage while blocking"
        if s2["p1Guard"] < s["p1Guard"] or (s["p1Guard"] == 0 and s2["p1Hitstun"] == 30 and broke_at is None
                                             and s2["p1Move"] in (GUARD_M, GUARD_STAND, GUARD_CROUCH)):
            events.append((t, int(s["p1Guard"]), int(s2["p1Guard"]), int(s2["p1Move"]), int(s2["p1Hitstun"]),
                           float(out["reward"][0]), int(s2["p2Move"])))
            if s["p1Guard"] == 0:
                broke_at = t
        if broke_at is not None and s2["p1Move"] == GUARD_BREAK:
            saw_guard_break_action = True
            break
        last = s2
    assert [(e[1], e[2]) for e in events[:3]] == [(3, 2), (2, 1), (1, 0)], events
    # the row of the attack that landed (P2's action, frozen in its hit-stop): guardAction and
    # guardStun, or guardBreakStun on the fourth hit (F:370-384, 446-454; ATK:14-54)
    row = {N_ATTACK: (GUARD_CROUCH, 12), N_SPECIAL: (GUARD_M, 15)}
    for e in events[:3]:
        assert e[6] in row and (e[3], e[4]) == row[e[6]] and e[5] == -0.3, e
    assert broke_at is not None and events[3][6] in row, events
    assert (events[3][3], events[3][4], events[3][5]) == (row[events[3][6]][0], 30, 0.0), events
    assert saw_guard_break_action
    assert last is not None


PUSH_W = F32(1.4)  # F00.asset basePushBoxRect width (every walking action's pushbox uses the base rect)


def kat_push_character(backend):
    """Both fighters walk forward into each other (P1 Right, P2 Left) for 60 frames.  Each tick
    moves them (F:300) and rebuilds the pushboxes at their positions (F:686-697, Rect x = position),
    then UpdatePushCharacterVsCharacter (BC:483-501) tests the Rects (Overlaps strict:
    r2.xMax > r1.xMin && r2.xMin < r1.xMax, xMax = width + x) and moves P1 by
    (r1.xMax - r2.xMin) * -1 / 2 and P2 by (r1.xMax - r2.xMin) * 1 / 2 (BC:490-494), so once
    they touch they stay pressed together, re-pushed every frame."""
    st, _ = run(backend, lambda t: R, lambda t: L, 60)
    x1, x2 = F32(-2), F32(2)
    step = F32(F32(F32(2.2) * F32(1)) * DT)
    contact = None
    for t, s in st:
        x1 = F32(x1 + step)
        x2 = F32(x2 + F32(F32(F32(2.2) * F32(-1)) * DT))
        r1_xmax, r2_xmax = F32(PUSH_W + x1), F32(PUSH_W + x2)
        if r2_xmax > x1 and x2 < r1_xmax and x1 < x2:
            d = F32(r1_xmax - x2)
            x1 = F32(x1 + F32(F32(d * F32(-1)) / F32(2)))
            x2 = F32(x2 + F32(F32(d * F32(1)) / F32(2)))
            contact = t if contact is None else contact
        assert s["p1Move"] == FORWARD and s["p2Move"] == FORWARD, t
        assert s["p1Position"] == x1 and s["p2Position"] == x2, (t, s["p1Position"], x1, s["p2Position"], x2)
    assert contact is not None and contact < 40, contact  # they met and kept being pushed apart


def kat_push_stage(backend):
    """P1 walks backward (Left) into the stage edge for 120 frames.  The pushbox as a BoxBase
    is centred on the position: xMin = rect.x - rect.width / 2 (F:12); UpdatePushCharacterVsBackground
    (BC:503-519) shifts the fighter by stageMinX - xMin whenever xMin < stageMinX = 10 * -1 / 2
    (BattleScene battleAreaWidth 10), so P1 ends pinned with its pushbox at the wall."""
    st, _ = run(backend, lambda t: L, lambda t: 0, 120)
    x = F32(-2)
    back = F32(F32(F32(1.8) * F32(1)) * DT)
    half = F32(PUSH_W / F32(2))
    stage_min = F32(F32(10) * F32(-1) / F32(2))
    pinned = 0
    for t, s in st:
        x = F32(x - back)
        xmin = F32(x - half)
        if xmin < stage_min:
            x = F32(x + F32(stage_min - xmin))
            pinned += 1
        assert s["p1Move"] == BACKWARD, t
        assert s["p1Position"] == x, (t, s["p1Position"], x)
        assert s["p2Position"] == F32(2)
    assert pinned > 10, pinned


ALL = {
    "idle": kat_idle, "walk": kat_walk, "n_attack_whiff": kat_n_attack_whiff, "dash_forward": kat_dash_forward,
    "dash_backward": kat_dash_backward, "charge_59": lambda b: kat_charge_special(b, 59),
    "charge_58": lambda b: kat_charge_special(b, 58), "charge_80": lambda b: kat_charge_special(b, 80),
    "proximity_guard": lambda b: kat_proximity_guard(b, True),
    "no_proximity_guard": lambda b: kat_proximity_guard(b, False), "guard_break": kat_guard_break,
    "recording_cap": kat_recording_cap, "push_character": kat_push_character, "push_stage": kat_push_stage,
}
