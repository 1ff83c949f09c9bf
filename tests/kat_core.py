"""Hand-derived known-answer scenarios for the simulation-core paths that, until round 4, only
kernel == oracle lockstep covered (VERDICT r03 "missing #1"):

* B_SPECIAL's overlapping movement windows, first match wins (ACT/B_SPECIAL.asset:14-83;
  ActionData.GetMovementData, AD:150-161; UpdateMovement F:291-319);
* the dash parsers at the edge of dashAllowFrame = 9 (F:585-635): a second tap 8 frames after
  the first dashes and 9 does not; a first press held 8 frames dashes and 9 does not (the inner
  scan wants a neutral input within the 8 frames before the press's last frame); a backward
  input in between cancels; P2's parse is facing-relative;
* the Intro tick's stale input (BC:183-200, 329-345; GetP1InputData BC:384-410): after RESET
  the remote actor's last input enters the cleared history (SetupBattleStart's ClearInput,
  F:120-135) before the first Fight frame, so a held Attack is no press on that frame, counts
  toward the 59-frame charge, and a held direction counts toward a dash;
* the execute-window buffer (RequestAction F:472-510, UpdateActionRequest F:212-229): an
  execute-window match only sets bufferActionID; the buffered action starts on a later tick,
  the first one with hitstun 0 and a landed hit (canCancelAttack F:531-539), never after a whiff;
* a hit landing on GUARD_PROXIMITY (NotifyDamaged F:357-398: Type Guard -> guardAction; AD:60-66,
  ACT/GUARD_PROXIMITY.asset type 3), reached through the proximity latch (F:262-285, 400-406);
* the reserved GUARD_BREAK taken exactly on the tick the stun reaches 0 (F:212-218, 373-379).

As in tests/kat_scenarios.py and tests/kat_combat.py, every expected value is derived here from
data/f00.json (the reference's F00 assets, re-extracted byte-identically by tests/test_tables.py)
and the cited C#, with numpy float32 arithmetic in the C# operand order -- never from the oracle
or the kernel.  A backend has ``reset()``, ``step(p1[1], p2[1]) -> outputs``, ``env_state()``,
``state()`` and ``set_state(records)`` (kat_combat.OracleKat on the CPU, gpu_backend.SimBackend
through the HIP path); scenarios run with dense rewards and same-step auto-reset.

Citations: BC = Assets/Script/BattleCore.cs, F = Assets/Script/Fighter.cs, AD =
Assets/Script/ActionData.cs, ACT = Assets/Fighter/F00/Actions/*.asset, ATK =
Assets/Fighter/F00/F00_AttackDataContainer.asset.
"""
import numpy as np

from tests.kat_combat import ACTIONS, ATTACKS, DT, F32, approach, load, run, step_x, velocity

L, R, A = 1, 2, 4
STAND, FORWARD, BACKWARD, DASH_F, DASH_B = 0, 1, 2, 10, 11
N_ATTACK, N_SPECIAL, B_SPECIAL = 100, 110, 115
GUARD_CROUCH, GUARD_BREAK, GUARD_PROX = 306, 310, 350
FIGHTER = {"dash_allow_frame": 9}  # checked against data/f00.json below


def _fighter_data():
    import json
    import os
    d = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "f00.json")))
    return d["fighter"]


def _a(x):
    return np.array([x], np.uint8)


def fresh(backend):
    """A reset whose Intro tick sees no stale input: one neutral step first, so both remote
    actors' current inputs (TrainingRemoteActor.input) are 0 when RESET runs the Intro tick."""
    backend.step(_a(0), _a(0))
    backend.reset()


def last_match_velocity(action, frame):
    """The *last* movement window holding the frame -- what GetMovementData does NOT do; used to
    show that a scenario tells the two apart."""
    v = 0.0
    for m in ACTIONS[action]["movements"]:
        if m["win"][0] <= frame <= m["win"][1]:
            v = m["velocity_x"]
    return v


# ---------------------------------------------------------------------------------------------
# B_SPECIAL: overlapping movement windows, first match
# ---------------------------------------------------------------------------------------------
def kat_b_special_windows(backend):
    """B_SPECIAL's movement windows overlap: [0,2] -> 3, [0,10] -> 2, [10,15] -> 1, [16] -> 0
    (ACT/B_SPECIAL.asset, in list order).  GetMovementData returns the first window that holds
    the frame (AD:150-161), so frames 0-2 move at 3, 3-10 at 2 (frame 10 too, although [10,15]
    also holds it), 11-15 at 1, frame 16 has velocity 0 (no move, F:314-317) and 17-54 no window.
    P1 charges Attack 59 frames (F:569-583) and releases with forward held: B_SPECIAL (F:234-238)
    from the release tick; P1 faces right, so x += v * 1 * dt per frame (F:316)."""
    mv = ACTIONS[B_SPECIAL]["movements"]
    assert [m["win"] for m in mv] == [[0, 2], [0, 10], [10, 15], [16, 16]]
    assert velocity(B_SPECIAL, 10) == 2.0 and last_match_velocity(B_SPECIAL, 10) == 1.0
    assert velocity(B_SPECIAL, 1) == 3.0 and last_match_velocity(B_SPECIAL, 1) == 2.0
    fresh(backend)
    rel = 59

    def p1(t):
        return A if t < rel else (R if t == rel else 0)
    st, _ = run(backend, p1, lambda t: 0, rel + 30)
    assert st[rel - 1]["p1Move"] == STAND and st[rel - 1]["p1Position"] == F32(-2)
    x = F32(-2)
    for f in range(30):
        t = rel + f
        x = step_x(x, velocity(B_SPECIAL, f), 1)
        s = st[t]
        assert (s["p1Move"], s["p1MoveFrame"]) == (B_SPECIAL, f), (f, s["p1Move"], s["p1MoveFrame"])
        assert s["p1Position"] == x, (f, s["p1Position"], x)
        assert s["p2Position"] == F32(2) and s["p2Move"] == STAND
    # the positions tell first match from last match: from the same frame-9 position, frame 10
    # moves by 2 * dt (window [0,10]), where the last matching window ([10,15]) would move 1 * dt
    x9 = st[rel + 9]["p1Position"]
    assert st[rel + 10]["p1Position"] == step_x(x9, 2.0, 1) != step_x(x9, last_match_velocity(B_SPECIAL, 10), 1)
    assert st[rel + 16]["p1Position"] == st[rel + 15]["p1Position"]  # velocity 0: no move
    assert st[rel + 20]["p1Position"] == st[rel + 16]["p1Position"]  # no window past 16


# ---------------------------------------------------------------------------------------------
# dash parsers at dashAllowFrame
# ---------------------------------------------------------------------------------------------
def _dash_case(backend, seq1, seq2, n):
    fresh(backend)
    st, _ = run(backend, lambda t: seq1[t] if t < len(seq1) else 0, lambda t: seq2[t] if t < len(seq2) else 0, n)
    return st


def _walk_then(x, seq, sign, fwd_bit, back_bit, until):
    """P's x over the scripted frames before the decisive one: a held forward / backward walks
    (FORWARD / BACKWARD from STAND, F:265-283; F:298-306), neutral frames stand still."""
    for t in range(until):
        a = seq[t] if t < len(seq) else 0
        if a & fwd_bit:
            x = step_x(x, 2.2, sign)
        elif a & back_bit:
            x = step_x(x, 1.8, sign, walk="backward")
    return x


def kat_dash_edges(backend):
    """CheckForwardDashInput / CheckBackwardDashInput (F:585-635) with dashAllowFrame 9 (F00.asset
    overrides FighterData's default 10): inputDown[0] must hold the direction; the scan looks at
    input[1..8] for the first directional input -- a backward one ends it (no dash), a forward one
    at i starts the inner scan of input[i+1 .. i+8] for a neutral input.  So, with the tap on the
    last frame of each script:
    * taps 8 frames apart dash, 9 apart do not (the first tap left the window);
    * a first press held 8 frames, released 1 frame, then tapped: dash (the inner scan reaches
      frame -1, the Intro tick's neutral input); held 9 frames: no dash (input[3..10] all forward);
    * forward, backward, forward on consecutive frames: input[1] is backward -> no dash;
    * the same for backward dashes, and for P2, whose forward is Left (F:642-666).
    The tap tick shows the dash at frame 0 moved by its frame-0 velocity (5 forward, -10
    backward, ACT/DASH_*.asset), or the walk it fell back to."""
    assert _fighter_data()["dash_allow_frame"] == FIGHTER["dash_allow_frame"] == 9
    vf0, vb0 = velocity(DASH_F, 0), velocity(DASH_B, 0)
    assert (vf0, vb0) == (5.0, -10.0)
    cases = []
    for gap, dash in ((8, True), (9, False), (1, False), (2, True)):  # gap 1: the press is held, no inputDown
        cases.append(("tap", gap, dash))
    for hold, dash in ((8, True), (9, False), (1, True)):
        cases.append(("hold", hold, dash))
    cases.append(("interrupt", 0, False))
    for who in (0, 1):  # P1 / P2
        fwd, back = (R, L) if who == 0 else (L, R)
        sign = 1 if who == 0 else -1
        for direction in ("forward", "backward"):
            d_in, o_in = (fwd, back) if direction == "forward" else (back, fwd)
            for kind, k, dash in cases:
                if kind == "tap":
                    seq = [d_in] + [0] * (k - 1) + [d_in] if k > 1 else [d_in, d_in]
                elif kind == "hold":
                    seq = [d_in] * k + [0, d_in]
                else:
                    seq = [d_in, o_in, d_in]
                tap = len(seq) - 1
                st = _dash_case(backend, seq if who == 0 else [], seq if who == 1 else [], tap + 1)
                s = st[tap]
                key = "p1" if who == 0 else "p2"
                x0 = F32(-2) if who == 0 else F32(2)
                x = _walk_then(x0, seq, sign, fwd, back, tap)
                label = (who, direction, kind, k)
                if dash:
                    act, x_exp = (DASH_F, step_x(x, vf0, sign)) if direction == "forward" else (DASH_B, step_x(x, vb0, sign))
                    assert (s[key + "Move"], s[key + "MoveFrame"]) == (act, 0), (label, s[key + "Move"])
                else:
                    act = FORWARD if direction == "forward" else BACKWARD
                    x_exp = step_x(x, 2.2, sign) if direction == "forward" else step_x(x, 1.8, sign, walk="backward")
                    assert s[key + "Move"] == act, (label, s[key + "Move"], s[key + "MoveFrame"])
                assert s[key + "Position"] == x_exp, (label, s[key + "Position"], x_exp)


# ---------------------------------------------------------------------------------------------
# the Intro tick's stale input
# ---------------------------------------------------------------------------------------------
def kat_intro_stale_input(backend):
    """FootsiesEnv.reset sends RESET (Stop -> Intro -> Fight, BC:143-146, 247-288).  The Intro tick
    (UpdateIntroState, BC:329-345) reads the actors' inputs like a Fight tick -- in training,
    TrainingRemoteActor.input, the last action the agent sent -- and feeds them to UpdateInput
    after SetupBattleStart cleared the history (F:120-135).  Fight then restarts the recording
    (BC:279-286), so state(-1) reports MostRecentAction 0.  Observable on the next frames:
    * Attack held into the reset: pressing Attack on the first Fight frame is no inputDown (F:184)
      -- P1 stays in STAND (frame 2: SetCurrentAction at Intro + two increments) instead of
      N_ATTACK -- and the Intro frame counts toward the charge: 58 Fight frames held and then
      released give N_SPECIAL (a fresh reset needs 59, tests/kat_scenarios.py charge_58);
    * Right held into the reset (P1's forward): neutral, then Right on the second Fight frame is a
      forward dash (forward found at input[2] = the Intro frame, neutral beyond it), where a
      fresh reset gives FORWARD."""
    # control: no stale input
    fresh(backend)
    s = backend.env_state()[0]
    assert (s["globalFrame"], s["p1MostRecentAction"], s["p1Move"], s["p1MoveFrame"]) == (-1, 0, STAND, 1)
    backend.step(_a(A), _a(0))
    assert backend.env_state()[0]["p1Move"] == N_ATTACK
    # Attack held into RESET
    fresh(backend)
    for _ in range(3):
        backend.step(_a(A), _a(0))
    backend.reset()
    s = backend.env_state()[0]
    assert (s["globalFrame"], s["p1MostRecentAction"], s["p1Move"], s["p1MoveFrame"]) == (-1, 0, STAND, 1)
    assert backend.state()[0]["f"][0]["attack_hold"] == 1  # the Intro frame's Attack
    st, out = run(backend, lambda t: A if t < 58 else 0, lambda t: 0, 59)
    assert (st[0]["p1Move"], st[0]["p1MoveFrame"]) == (STAND, 2) and out[0]["action"][0, 0] == A
    for t in range(1, 58):
        assert st[t]["p1Move"] == STAND, t
    assert (st[58]["p1Move"], st[58]["p1MoveFrame"]) == (N_SPECIAL, 0), st[58]["p1Move"]
    assert st[58]["p1Position"] == step_x(F32(-2), velocity(N_SPECIAL, 0), 1)
    # Right held into RESET: neutral, Right -> dash
    for stale, expect in ((R, DASH_F), (0, FORWARD)):
        fresh(backend)
        backend.step(_a(stale), _a(0))
        backend.reset()
        st, _ = run(backend, lambda t: R if t == 1 else 0, lambda t: 0, 2)
        assert st[0]["p1Move"] == STAND and st[0]["p1Position"] == F32(-2)
        assert st[1]["p1Move"] == expect, (stale, st[1]["p1Move"])
        v = velocity(DASH_F, 0) if expect == DASH_F else None
        x = step_x(F32(-2), v, 1) if v is not None else step_x(F32(-2), 2.2, 1)
        assert st[1]["p1Position"] == x


# ---------------------------------------------------------------------------------------------
# the execute-window buffer
# ---------------------------------------------------------------------------------------------
def kat_execute_window_buffer(backend):
    """N_ATTACK's cancel windows (ACT/N_ATTACK.asset): frames 1-3 buffer N_SPECIAL, 4-5 execute
    N_SPECIAL.  A second Attack press while N_ATTACK runs requests N_SPECIAL (F:241-246);
    RequestAction (F:472-510) on an execute-window match sets bufferActionID and returns true --
    it does not switch the action.  The buffer is taken by a later UpdateActionRequest
    (F:222-229) once canCancelAttack() (a landed hit: canCancelOnWhiff is false, F:531-539) and
    no hitstun.
    * Landed (the jab of kat_combat.kat_landed_n_attack: hit on frame 4 at tick 21, stun 12 on
      both, frames frozen): pressed on tick 33 -- the stun reached 0 in that tick's
      IncrementActionFrame (F:149-154), the frame is still 4 -- P1 stays N_ATTACK frame 4 with
      N_SPECIAL buffered, and N_SPECIAL starts at frame 0 on tick 34 (moving by its frame-0
      velocity 2, ACT/N_SPECIAL.asset).  Pressed on tick 32 (stun 1, frame 4): buffered; the
      early return needs hitstun <= 0, so N_SPECIAL starts on tick 33, the first tick at 0.
    * Whiffed (distance 4): pressed on N_ATTACK's frame 4: N_SPECIAL stays buffered, never taken
      (hit count 0); N_ATTACK runs its 22 frames and SetCurrentAction(STAND) clears the buffer."""
    assert ACTIONS[N_ATTACK]["cancels"] == [
        {"win": [1, 3], "buffer": True, "execute": False, "action_ids": [N_SPECIAL]},
        {"win": [4, 5], "buffer": False, "execute": True, "action_ids": [N_SPECIAL]}]
    x1, x2 = approach(17)
    for press, starts in ((33, 34), (32, 33)):
        fresh(backend)

        def p1(t, press=press):
            return R if t < 17 else (A if t in (17, press) else 0)
        st, _ = run(backend, p1, lambda t: L if t < 17 else 0, 17)
        assert (st[16]["p1Position"], st[16]["p2Position"]) == (x1, x2)
        states, bufs = {}, {}
        for t in range(17, starts + 2):
            backend.step(_a(p1(t)), _a(0))
            states[t] = backend.env_state()[0].copy()
            bufs[t] = int(backend.state()[0]["f"][0]["buffer_action_id"])
        h = states[21]
        assert (h["p1Move"], h["p1MoveFrame"], h["p1Hitstun"], h["p2Move"]) == (N_ATTACK, 4, 12, 200)
        for t in range(21, starts):
            assert (states[t]["p1Move"], states[t]["p1MoveFrame"]) == (N_ATTACK, 4), (press, t)
            assert states[t]["p1Hitstun"] == 12 - (t - 21), (press, t)
            assert bufs[t] == (N_SPECIAL if t >= press else -1), (press, t, bufs[t])
        s = states[starts]
        assert (s["p1Move"], s["p1MoveFrame"], s["p1Hitstun"]) == (N_SPECIAL, 0, 0), (press, s["p1Move"])
        assert s["p1Position"] == step_x(x1, velocity(N_SPECIAL, 0), 1) and bufs[starts] == -1
    # whiff: buffered on frame 4, never taken
    fresh(backend)
    bufs, st = {}, {}
    for t in range(24):
        backend.step(_a(A if t in (0, 4) else 0), _a(0))
        st[t] = backend.env_state()[0].copy()
        bufs[t] = int(backend.state()[0]["f"][0]["buffer_action_id"])
    for t in range(22):
        assert (st[t]["p1Move"], st[t]["p1MoveFrame"]) == (N_ATTACK, t), t
        assert bufs[t] == (N_SPECIAL if t >= 4 else -1), (t, bufs[t])
    assert st[22]["p1Move"] == STAND and bufs[22] == -1 and st[22]["p2Guard"] == 3


# ---------------------------------------------------------------------------------------------
# a hit on GUARD_PROXIMITY; the reserved GUARD_BREAK at stun 0
# ---------------------------------------------------------------------------------------------
def _proximity_guard_hit(backend, p1_guard, ticks):
    """Both walk in 17 frames (distance ~2.504); then P2 jabs and P1 holds back.  Tick 17: P1's
    request gives BACKWARD (the latch is still clear; F:273-279) and it steps back; P2's N_ATTACK
    frame-0 proximity hitbox ([x2 - 3, x2], ACT/N_ATTACK.asset rect x 1.5 w 3, facing left)
    overlaps P1's hurtbox, so NotifyInProximityGuardRange latches isReserveProximityGuard (P1's
    isInputBackward was set this tick; BC:583-586, F:400-406).  Ticks 18-20: back + latch ->
    GUARD_PROXIMITY (1 frame, always cancelable, re-requested as it ends), re-latched every tick
    by the proximity box; no movement.  Tick 21: N_ATTACK's real hitbox (frames 4-5,
    [x2 - 1.8, x2]) reaches P1's base hurtbox ([x1 - 0.75, x1 + 0.75])."""
    x1, x2 = approach(17)
    fresh(backend)
    run(backend, lambda t: R, lambda t: L, 17)
    if p1_guard != 3:
        s = backend.state()
        s["f"][0, 0]["guard"] = p1_guard
        backend.set_state(s)
    x1b = step_x(x1, 1.8, 1, walk="backward")
    assert x2 - F32(1.8) <= x1b + F32(0.75) and x2 - F32(3.0) <= x1b + F32(0.75)
    st, out, cs = {}, {}, {}
    for t in range(17, 17 + ticks):
        o = backend.step(_a(L), _a(A if t == 17 else 0))
        st[t] = backend.env_state()[0].copy()
        out[t] = {k: np.array(v, copy=True) for k, v in o.items()}
        cs[t] = backend.state()[0].copy()
    assert st[17]["p1Move"] == BACKWARD and st[17]["p1Position"] == x1b
    for t in (18, 19, 20):
        assert (st[t]["p1Move"], st[t]["p1MoveFrame"]) == (GUARD_PROX, 0), (t, st[t]["p1Move"])
        assert st[t]["p1Position"] == x1b and st[t]["p2MoveFrame"] == t - 17
    return st, out, cs, x1b


def kat_hit_on_guard_proximity(backend):
    """N_ATTACK lands on a fighter in GUARD_PROXIMITY: its Type is Guard (ACT/GUARD_PROXIMITY.asset
    type 3 = ActionType.Guard, AD:60-66), so NotifyDamaged blocks (F:370-384): guard 3 -> 2 (guard
    damage applies on every hit, F:360-368), no vital damage, SetCurrentAction(guardActionID) =
    GUARD_CROUCH (ATK N_ATTACK guardAction 306), result Guard -> guardStunFrame 12 on both
    fighters (BC:574-578, F:446-454).  Dense reward -0.3 (P1's guard dropped, FE:393-394).  When
    the stun is over, GUARD_CROUCH frame 0 pushes P1 back (velocity -2, ACT/GUARD_CROUCH.asset)."""
    atk = ATTACKS[1]
    assert (atk["guard_action"], atk["guard_stun"], atk["guard_damage"], atk["vital_damage"]) == (GUARD_CROUCH, 12, 1, 0)
    st, out, _, x1b = _proximity_guard_hit(backend, 3, 18)
    h = st[21]
    assert (h["p1Move"], h["p1MoveFrame"], h["p1Guard"], h["p1Vital"]) == (GUARD_CROUCH, 0, 2, 1), h["p1Move"]
    assert (h["p1Hitstun"], h["p2Hitstun"], h["p2Move"], h["p2MoveFrame"]) == (12, 12, N_ATTACK, 4)
    assert out[21]["reward"][0] == -0.3 and not out[21]["terminated"][0]
    for t in range(22, 33):
        assert (st[t]["p1Move"], st[t]["p1MoveFrame"], st[t]["p1Hitstun"]) == (GUARD_CROUCH, 0, 33 - t), t
        assert st[t]["p1Position"] == x1b, t
    assert st[33]["p1Hitstun"] == 0 and st[33]["p1Position"] == step_x(x1b, velocity(GUARD_CROUCH, 0), 1)
    assert st[34]["p1MoveFrame"] == 1


def kat_guard_break_reserve(backend):
    """The same hit with P1's guard loaded at 0 (STATE_LOAD): guard 0 - 1 < 0 is a guard break
    (F:362-367): guard stays 0, SetCurrentAction(GUARD_CROUCH) with reserveDamageActionID =
    GUARD_BREAK, result GuardBreak -> guardBreakStunFrame 30 on both (ATK N_ATTACK).  No guard
    dropped, so the dense reward is 0.  For ticks 22-50 the stun counts 29 .. 1 with the frame
    frozen; P1 keeps holding back, but UpdateActionRequest's reserve branch waits for hitstun <= 0
    (F:212-218) and GUARD_CROUCH cannot be cancelled into BACKWARD.  Tick 51: the stun reaches 0
    in IncrementActionFrame, and the same tick's UpdateActionRequest takes the reserve:
    GUARD_BREAK frame 0 (SetCurrentAction clears the reserve), which moves P1 by its frame-0
    velocity -2 (ACT/GUARD_BREAK.asset) in that tick's UpdateMovement."""
    assert ATTACKS[1]["guard_break_stun"] == 30
    st, out, cs, x1b = _proximity_guard_hit(backend, 0, 36)
    h = st[21]
    assert (h["p1Move"], h["p1MoveFrame"], h["p1Guard"], h["p1Vital"]) == (GUARD_CROUCH, 0, 0, 1), h["p1Move"]
    assert (h["p1Hitstun"], h["p2Hitstun"]) == (30, 30) and out[21]["reward"][0] == 0.0
    for t in range(21, 51):
        assert (st[t]["p1Move"], st[t]["p1MoveFrame"], st[t]["p1Hitstun"]) == (GUARD_CROUCH, 0, 51 - t), t
        assert int(cs[t]["f"][0]["reserve_action_id"]) == GUARD_BREAK, t
        assert st[t]["p1Position"] == x1b and (st[t]["p2Move"], st[t]["p2MoveFrame"]) == (N_ATTACK, 4), t
    s = st[51]
    assert (s["p1Move"], s["p1MoveFrame"], s["p1Hitstun"]) == (GUARD_BREAK, 0, 0), s["p1Move"]
    assert int(cs[51]["f"][0]["reserve_action_id"]) == -1
    assert s["p1Position"] == step_x(x1b, velocity(GUARD_BREAK, 0), 1)
    assert (s["p2Move"], s["p2MoveFrame"], s["p2Hitstun"]) == (N_ATTACK, 4, 0)
    assert (st[52]["p1Move"], st[52]["p1MoveFrame"]) == (GUARD_BREAK, 1) and st[52]["p2MoveFrame"] == 5


# ---------------------------------------------------------------------------------------------
# the attack table's row for every attack: blocked, landed, guard broken
# ---------------------------------------------------------------------------------------------
B_ATTACK, DAMAGE, GUARD_M, GUARD_STAND = 105, 200, 301, 305
HALF_HURT = F32(0.75)  # F00.asset baseHurtBoxRect width 1.5, a centred BoxBase (F:8-26)
PUSH_W = F32(1.4)      # F00.asset basePushBoxRect width, a Rect whose x is the left edge (BC:483-501)
# attacker action -> (attack ID of its real hitbox, the frame loaded: the one before the box is out)
ATTACK_OF = {N_ATTACK: (1, 3), B_ATTACK: (2, 2), N_SPECIAL: (10, 10), B_SPECIAL: (11, 1)}


def _real_hitbox(action, frame):
    boxes = [h for h in ACTIONS[action]["hitboxes"] if not h["proximity"] and h["win"][0] <= frame <= h["win"][1]]
    assert len(boxes) == 1, (action, frame)
    return boxes[0]


def _table_hit(backend, attacker, action, guard, block, gap):
    """One arena loaded (STATE_LOAD) with the attacker in `action` one frame before its real
    hitbox comes out and the defender standing `gap` apart, holding back when `block` (its back
    is away from the attacker: P1 Left, P2 Right; F:642-666) with its guard loaded at `guard`.
    Tick 0: the attacker's frame advances into the hitbox window and it moves by that frame's
    velocity (N_SPECIAL 5, B_SPECIAL 3, the attacks none); a blocking defender walks back
    (STAND -> BACKWARD, always cancelable, F:265-283) by 1.8 * dt; the pushboxes stay apart and
    the real hitbox reaches the base hurtbox (checked here in float32), so NotifyDamaged runs on
    tick 0.  Returns per-tick env states, outputs and canonical states, and both x after tick 0."""
    atk_id, f0 = ATTACK_OF[action]
    hb = _real_hitbox(action, f0 + 1)
    assert hb["attack_id"] == atk_id
    a_sign = 1 if attacker == 0 else -1         # P1 faces right, P2 left
    xa = F32(-a_sign * gap / 2)
    xd = F32(a_sign * gap / 2)
    fresh(backend)
    atk_rec, def_rec = (action, f0), (STAND, 0)
    p1, p2 = ((xa,) + atk_rec, (xd,) + def_rec) if attacker == 0 else ((xd,) + def_rec, (xa,) + atk_rec)
    load(backend, p1, p2)
    if guard != 3:
        s = backend.state()
        s["f"][0, 1 - attacker]["guard"] = guard
        backend.set_state(s)
    xa1 = step_x(xa, velocity(action, f0 + 1), a_sign)
    xd1 = step_x(xd, 1.8, -a_sign, walk="backward") if block else xd
    c = F32(xa1 + F32(F32(hb["rect"][0]) * F32(a_sign)))
    lo, hi = F32(c - F32(F32(hb["rect"][2]) / F32(2))), F32(c + F32(F32(hb["rect"][2]) / F32(2)))
    assert lo <= F32(xd1 + HALF_HURT) and F32(xd1 - HALF_HURT) <= hi, (action, lo, hi, xd1)
    left, right = (xa1, xd1) if attacker == 0 else (xd1, xa1)
    assert F32(left + PUSH_W) < right  # no character push (strict Rect overlap, BC:485-499)
    back = R if attacker == 0 else L  # the defender's back: P2's is Right, P1's Left
    d_in = back if block else 0
    ins = (lambda t: 0, lambda t: d_in) if attacker == 0 else (lambda t: d_in, lambda t: 0)
    st, out, cs = {}, {}, {}
    for t in range(40):
        o = backend.step(_a(ins[0](t)), _a(ins[1](t)))
        st[t] = backend.env_state()[0].copy()
        out[t] = {k: np.array(v, copy=True) for k, v in o.items()}
        cs[t] = backend.state()[0].copy()
        if o["terminated"][0]:
            break
    return st, out, cs, xa1, xd1


def kat_attack_table_rows(backend):
    """F:446-454 picks the stun from the attacker's AttackData row by DamageResult, and NotifyDamaged
    (F:357-398) the defender's action from the same row (ATK:14-54):

      attack      damageAction  guardAction  hitStun  guardStun  guardBreakStun  vital dmg
      N_ATTACK 1      200          306          12       12           30            0
      B_ATTACK 2      200          305          12       12           30            0
      N_SPECIAL 10    500          301           0       15           30            1
      B_SPECIAL 11    500          301           0       15           30            1

    For each attack, attacking as P1 and as P2 (the collision's two trade phases, BC:523-586):
    * blocked (the defender walks back, BACKWARD counts as blocking, F:370-371): guard 3 -> 2,
      guardAction at frame 0, guardStun on both fighters, dense reward -0.3 / +0.3 for the
      defender's guard (FE:393-394), vital kept; the stun counts down with both frames frozen
      (F:149-154) and, on the tick it reaches 0, the defender moves by its guard action's frame-0
      velocity (ACT/GUARD_*.asset) away from the attacker;
    * guard broken (guard loaded at 0, blocking): guard stays 0, guardAction with GUARD_BREAK
      reserved, guardBreakStun 30 on both, reward 0; on the tick the stun reaches 0 the reserve
      is taken (F:212-218): GUARD_BREAK frame 0;
    * landed (standing): the attacks give DAMAGE with hitStun 12 and guard 3 -> 2 (guard damage
      applies unblocked too); the specials kill: DEAD, terminated, the episode's return +-1 with
      the guard drop included (FE:388-405), hitStun 0 on both;
    * landed on a guard of 0 (isGuardBreak set, but not blocking): the damage branch, DAMAGE with
      hitStun 12 -- never the guard-break stun -- and reward 0."""
    guard_row = {N_ATTACK: GUARD_CROUCH, B_ATTACK: GUARD_STAND, N_SPECIAL: GUARD_M, B_SPECIAL: GUARD_M}
    for action, (atk_id, _) in ATTACK_OF.items():
        a = ATTACKS[atk_id]
        assert a["guard_action"] == guard_row[action] and a["guard_damage"] == 1 and a["guard_break_stun"] == 30
        assert (a["damage_action"], a["hit_stun"], a["guard_stun"], a["vital_damage"]) == (
            (DAMAGE, 12, 12, 0) if action in (N_ATTACK, B_ATTACK) else (500, 0, 15, 1)), action
        special = action in (N_SPECIAL, B_SPECIAL)
        gap = 1.6 if action == B_SPECIAL else 2.0
        for attacker in (0, 1):
            A_, D_ = ("p1", "p2") if attacker == 0 else ("p2", "p1")
            sgn = 1.0 if attacker == 0 else -1.0  # dense reward: + when P2's guard drops
            dsign = -1 if attacker == 0 else 1    # the defender's facing sign
            label = (action, attacker)
            # blocked
            st, out, cs, xa1, xd1 = _table_hit(backend, attacker, action, 3, True, gap)
            h, stun = st[0], a["guard_stun"]
            assert (h[D_ + "Move"], h[D_ + "MoveFrame"], h[D_ + "Guard"], h[D_ + "Vital"]) == (
                a["guard_action"], 0, 2, 1), (label, h[D_ + "Move"], h[D_ + "Guard"])
            assert (h[A_ + "Move"], h[A_ + "MoveFrame"]) == (action, ATTACK_OF[action][1] + 1), label
            assert (h[A_ + "Hitstun"], h[D_ + "Hitstun"]) == (stun, stun), (label, h[A_ + "Hitstun"])
            assert out[0]["reward"][0] == sgn * 0.3 and not out[0]["terminated"][0], label
            assert h[D_ + "Position"] == xd1 and h[A_ + "Position"] == xa1, label
            for t in range(1, stun):
                s = st[t]
                assert (s[D_ + "Move"], s[D_ + "MoveFrame"], s[D_ + "Hitstun"]) == (a["guard_action"], 0, stun - t), (label, t)
                assert (s[A_ + "MoveFrame"], s[A_ + "Hitstun"]) == (ATTACK_OF[action][1] + 1, stun - t), (label, t)
                assert s[D_ + "Position"] == xd1, (label, t)
            s = st[stun]
            assert s[D_ + "Hitstun"] == 0 and s[D_ + "Position"] == step_x(xd1, velocity(a["guard_action"], 0), dsign), label
            # guard broken
            st, out, cs, xa1, xd1 = _table_hit(backend, attacker, action, 0, True, gap)
            h = st[0]
            assert (h[D_ + "Move"], h[D_ + "MoveFrame"], h[D_ + "Guard"], h[D_ + "Vital"]) == (
                a["guard_action"], 0, 0, 1), (label, h[D_ + "Move"])
            assert (h[A_ + "Hitstun"], h[D_ + "Hitstun"]) == (30, 30) and out[0]["reward"][0] == 0.0, label
            assert int(cs[0]["f"][1 - attacker]["reserve_action_id"]) == GUARD_BREAK, label
            for t in range(1, 30):
                assert (st[t][D_ + "Move"], st[t][D_ + "Hitstun"]) == (a["guard_action"], 30 - t), (label, t)
            s = st[30]
            assert (s[D_ + "Move"], s[D_ + "MoveFrame"], s[D_ + "Hitstun"]) == (GUARD_BREAK, 0, 0), (label, s[D_ + "Move"])
            assert s[D_ + "Position"] == step_x(xd1, velocity(GUARD_BREAK, 0), dsign), label
            # landed, then landed on a guard of 0
            for guard in (3, 0):
                st, out, cs, xa1, xd1 = _table_hit(backend, attacker, action, guard, False, gap)
                o = out[0]
                if special:  # vital 1 -> 0: DEAD, the battle is over this tick (BC:212-218)
                    assert o["terminated"][0] == 1, (label, guard)
                    r0 = sgn * 0.3 if guard else 0.0  # FE:393-404 in its float64 order
                    assert o["reward"][0] == r0 + (sgn * 1.0 - r0), (label, guard, o["reward"][0])
                    dk = 0 if attacker == 1 else 1
                    assert o["final_move"][0, dk] == 0 and o["final_guard"][0, dk] == (2 if guard else 0), (label, guard)
                    assert tuple(o["final_hitstun"][0]) == (0, 0), (label, guard)  # hitStun 0
                    continue
                h = st[0]
                assert (h[D_ + "Move"], h[D_ + "MoveFrame"], h[D_ + "Vital"]) == (DAMAGE, 0, 1), (label, guard, h[D_ + "Move"])
                assert h[D_ + "Guard"] == (2 if guard else 0) and (h[A_ + "Hitstun"], h[D_ + "Hitstun"]) == (12, 12), (label, guard)
                assert out[0]["reward"][0] == (sgn * 0.3 if guard else 0.0) and not o["terminated"][0], (label, guard)
                assert int(cs[0]["f"][1 - attacker]["reserve_action_id"]) == -1, (label, guard)
                s = st[12]
                assert (s[D_ + "Move"], s[D_ + "Hitstun"]) == (DAMAGE, 0), (label, guard)
                assert s[D_ + "Position"] == step_x(xd1, velocity(DAMAGE, 0), dsign), (label, guard)


# ---------------------------------------------------------------------------------------------
# UpdateActionRequest's request order and RequestAction's rules, from inputs
# ---------------------------------------------------------------------------------------------
def kat_request_chain(backend):
    """UpdateActionRequest (F:201-286) requests, in order: the special or the attack, the dash,
    then the movement; RequestAction (F:472-510) sets an action when the current one has ended
    (isActionEnd: frame >= frameCount, F:90), never re-sets the current action, and otherwise only
    from an always-cancelable action or through a cancel window.  Hand-derived from data/f00.json:
    * Attack pressed with a direction held (forward, backward or both; P2's forward is Left) is
      B_ATTACK, without one N_ATTACK (F:247-253); the movement request after it finds B_ATTACK at
      frame 0 with no cancel window and does nothing, and B_ATTACK has no movement: x stays;
    * FORWARD held for 50 ticks: the same-action request is refused, so the frame counts 0 .. 23;
      on the tick it reaches frameCount 24 the action has ended and FORWARD is set again at 0
      (frames 0..23, 0..23, 0, 1), walking every tick;
    * N_ATTACK pressed again: on frame 21 (not ended) the press requests N_SPECIAL (F:243-246),
      which no window of frame 21 takes -- nothing happens and STAND follows on frame 22; on the
      tick its frame reaches 22 (ended) the press requests N_ATTACK, which is set at frame 0;
    * a forward tap, a neutral frame, then forward + Attack: the dash input is there (taps two
      frames apart), but B_ATTACK is requested first and the dash request that follows finds
      B_ATTACK at frame 0 with no cancel window (F:256-259): B_ATTACK, no dash;
    * B_ATTACK's execute window (frames 3-5, N_SPECIAL): Attack pressed on the tick B_ATTACK's real
      hitbox lands (frame 3) buffers N_SPECIAL; the hit stuns both for 12 (ATK B_ATTACK); on the
      tick the stun reaches 0 the buffer is taken (a landed hit: canCancelAttack, F:222-229):
      N_SPECIAL frame 0, moving by its frame-0 velocity 2."""
    fwd_speed = _fighter_data()["forward_move_speed"]
    assert ACTIONS[FORWARD]["frame_count"] == 24 and ACTIONS[FORWARD]["always_cancelable"]
    assert ACTIONS[N_ATTACK]["frame_count"] == 22 and not ACTIONS[B_ATTACK]["movements"]
    assert ACTIONS[B_ATTACK]["cancels"] == [
        {"win": [1, 2], "buffer": True, "execute": False, "action_ids": [N_SPECIAL]},
        {"win": [3, 5], "buffer": False, "execute": True, "action_ids": [N_SPECIAL]}]
    # Attack with / without a direction, both players
    for who in (0, 1):
        for d, act in ((0, N_ATTACK), (R, B_ATTACK), (L, B_ATTACK), (L | R, B_ATTACK)):
            fresh(backend)
            backend.step(_a(A | d if who == 0 else 0), _a(A | d if who == 1 else 0))
            s = backend.env_state()[0]
            key = "p1" if who == 0 else "p2"
            assert (s[key + "Move"], s[key + "MoveFrame"]) == (act, 0), (who, d, s[key + "Move"])
            assert s[key + "Position"] == (F32(-2) if who == 0 else F32(2)), (who, d)
    # FORWARD held: the frame cycles through 0..23
    fresh(backend)
    st, _ = run(backend, lambda t: R, lambda t: 0, 50)
    x = F32(-2)
    for t in range(50):
        x = step_x(x, fwd_speed, 1)
        assert (st[t]["p1Move"], st[t]["p1MoveFrame"]) == (FORWARD, t % 24), (t, st[t]["p1MoveFrame"])
        assert st[t]["p1Position"] == x, t
    # N_ATTACK pressed again on frame 21 / on the tick it ends (frame 22)
    for press, expect in ((21, (N_ATTACK, 21, STAND, 0)), (22, (N_ATTACK, 21, N_ATTACK, 0))):
        fresh(backend)
        st, _ = run(backend, lambda t, press=press: A if t in (0, press) else 0, lambda t: 0, 23)
        assert (st[21]["p1Move"], st[21]["p1MoveFrame"], st[22]["p1Move"], st[22]["p1MoveFrame"]) == expect, press
        assert all((st[t]["p1Move"], st[t]["p1MoveFrame"]) == (N_ATTACK, t) for t in range(21)), press
    # the attack request comes before the dash request
    fresh(backend)
    st, _ = run(backend, lambda t: (R, 0, R | A)[t], lambda t: 0, 3)
    assert [st[t]["p1Move"] for t in range(3)] == [FORWARD, STAND, B_ATTACK], [st[t]["p1Move"] for t in range(3)]
    assert st[2]["p1MoveFrame"] == 0 and st[2]["p1Position"] == step_x(F32(-2), fwd_speed, 1)
    # B_ATTACK -> N_SPECIAL through the execute window after a landed hit (P1 loaded at frame 2,
    # P2 standing 2.0 away: the real hitbox [x1, x1 + 1.6] reaches P2's hurtbox [0.25, 1.75])
    fresh(backend)
    load(backend, (-1.0, B_ATTACK, 2), (1.0, STAND, 0))
    st, _ = run(backend, lambda t: A if t == 0 else 0, lambda t: 0, 14)
    h = st[0]
    assert (h["p1Move"], h["p1MoveFrame"], h["p2Move"], h["p1Hitstun"], h["p2Hitstun"]) == (B_ATTACK, 3, DAMAGE, 12, 12)
    assert int(backend.state()[0]["f"][0]["buffer_action_id"]) == -1  # (taken by tick 12, see below)
    for t in range(1, 12):
        assert (st[t]["p1Move"], st[t]["p1MoveFrame"], st[t]["p1Hitstun"]) == (B_ATTACK, 3, 12 - t), t
    s = st[12]
    assert (s["p1Move"], s["p1MoveFrame"], s["p1Hitstun"]) == (N_SPECIAL, 0, 0), s["p1Move"]
    assert s["p1Position"] == step_x(F32(-1.0), velocity(N_SPECIAL, 0), 1)
    assert (st[13]["p1Move"], st[13]["p1MoveFrame"]) == (N_SPECIAL, 1)


ALL = {
    "attack_table_rows": kat_attack_table_rows,
    "request_chain": kat_request_chain,
    "b_special_windows": kat_b_special_windows,
    "dash_edges": kat_dash_edges,
    "intro_stale_input": kat_intro_stale_input,
    "execute_window_buffer": kat_execute_window_buffer,
    "hit_on_guard_proximity": kat_hit_on_guard_proximity,
    "guard_break_reserve": kat_guard_break_reserve,
}

# The C# paths each scenario pins (DESIGN.md section 3 reproduces this table)
PINS = {
    "request_chain": "F:201-286 request order (special / attack, dash, movement), F:472-510 ended / same-action / "
                     "cancel-window rules, B_ATTACK's execute window taken at stun 0 after a hit (F:222-229)",
    "attack_table_rows": "F:357-398, 446-454 + ATK:14-54: every attack's guardAction / guardStun, damageAction / hitStun, "
                         "guardBreakStun with GUARD_BREAK reserved, as P1 and as P2 (BC:523-586)",
    "b_special_windows": "AD:150-161 first-match GetMovementData over ACT/B_SPECIAL.asset:14-83's overlapping windows",
    "dash_edges": "F:585-635 dash parsers at dashAllowFrame 9 (tap gap 8/9, hold 8/9, interrupt, P2 facing)",
    "intro_stale_input": "BC:183-200, 329-345 Intro tick input after SetupBattleStart's ClearInput (F:120-135)",
    "execute_window_buffer": "F:472-510 execute window -> bufferActionID; F:212-229, 531-539 taken at stun 0 after a hit",
    "hit_on_guard_proximity": "F:357-398 Type Guard -> guardAction (AD:60-66), latch F:262-285, 400-406",
    "guard_break_reserve": "F:212-218, 362-379 reserved GUARD_BREAK taken on the tick hitstun reaches 0",
}
