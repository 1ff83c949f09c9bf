"""Hand-derived known-answer scenarios for the general-geometry tick: fighters loaded off the
ground (position.y != 0) or with a flipped facing, which Fighter.LoadState restores
(Fighter.cs:741-744) although the game itself never produces them (SetupBattleStart F:120-135
puts both on y = 0 facing each other, and nothing turns a fighter or moves y on its own).

* a flipped fighter reads its inputs, walks and builds its boxes mirrored (IsForwardInput /
  IsBackwardInput F:642-666, UpdateMovement F:291-319, TransformToFightRect F:706-719);
* a fighter above its opponent's pushbox is not pushed (Rect.Overlaps tests y too, BC:483-488);
* every push adds the pushed fighter's y to itself -- UpdatePushCharacterVsBackground passes
  f.position.y as the y shift (BC:511-515), UpdatePushCharacterVsCharacter passes fighter1's /
  fighter2's own y when fighter1 is on the left, and fighter1's (already shifted) y to both when
  it is on the right (BC:491-498); ApplyPositionChange adds it to position.y and every box
  (F:331-350);
* a hitbox reaches a hurtbox only where their y ranges meet, inclusively (BoxBase.Overlaps
  F:17-25, yMax = y + height): an N_ATTACK hitbox [0, 0.3] hits a hurtbox from y = 0.3 down to
  y + 1.2 = 0, and misses at 0.31 or -1.21.

Expected values come from data/f00.json and the cited C# in numpy float32, never from the
oracle or the kernel.  The backend interface is tests/kat_core.py's.  BC =
Assets/Script/BattleCore.cs, F = Assets/Script/Fighter.cs, ACT = Assets/Fighter/F00/Actions.
"""
import numpy as np

from tests.kat_combat import ACTIONS, ATTACKS, DT, F32, _DATA, step_x
from tests.kat_core import fresh

L, R = 1, 2
STAND, FORWARD, BACKWARD, N_ATTACK, DAMAGE = 0, 1, 2, 100, 200
FD = _DATA["fighter"]
STAGE = F32(_DATA["stage"]["battle_area_width"] / 2)
PUSH_W = F32(FD["base_pushbox"][2])    # STAND / N_ATTACK use the base pushbox (useBaseRect)
PUSH_H = F32(FD["base_pushbox"][3])


def _a(x):
    return np.array([x], np.uint8)


def load_geom(backend, p1, p2):
    """STATE_LOAD of one arena in the Fight state; each fighter as a dict (x, act, frame, y, flip)."""
    s = backend.state()
    s["frame_count"] = 100
    s["recording_count"] = 100
    s["has_terminated"] = 0
    s["reset_pending"] = 0
    for k, d in enumerate((p1, p2)):
        f = s["f"][0, k]
        f["position_x"] = F32(d["x"])
        f["position_y"] = F32(d.get("y", 0.0))
        f["facing_flipped"] = int(d.get("flip", 0))
        f["action_id"] = d.get("act", STAND)
        f["action_frame"] = d.get("frame", 0)
        f["vital"], f["guard"], f["hit_count"], f["hitstun"] = 1, 3, 0, 0
        f["buffer_action_id"] = f["reserve_action_id"] = -1
        f["input_dir_history"] = 0
        f["attack_hold"] = 0
        f["is_input_backward"] = f["is_reserve_proximity_guard"] = f["has_won"] = 0
    backend.set_state(s)


def kat_flipped_walk(backend):
    """P1 loaded facing left (isFaceRight false) holds Right: for a left-facing fighter Right is
    the backward input (F:655-666), so STAND requests BACKWARD (F:265-283) and UpdateMovement
    moves it by -backwardMoveSpeed * sign * dt with sign = -1, i.e. to the right at 1.8 units/s
    (F:303-306).  Facing right, the same input walks FORWARD at 2.2 units/s.  The saved history is
    raw Left/Right bits whatever the facing: six frames of Right = 0b101010101010."""
    for flip, act, speed, walk in ((1, BACKWARD, FD["backward_move_speed"], "backward"),
                                   (0, FORWARD, FD["forward_move_speed"], None)):
        fresh(backend)
        load_geom(backend, {"x": -2.0, "flip": flip}, {"x": 2.0})
        x = F32(-2.0)
        sign = -1 if flip else 1
        for t in range(6):
            backend.step(_a(R), _a(0))
            s = backend.env_state()[0]
            x = step_x(x, speed, sign, walk=walk)
            assert s["p1Move"] == act and s["p1Position"] == x, (flip, t, s["p1Move"], s["p1Position"], x)
        f = backend.state()[0]["f"][0]
        assert f["facing_flipped"] == flip and f["input_dir_history"] == 0b101010101010
    # the walk really went right in both cases, at the two speeds
    assert x > F32(-2.0)


def _push_pair(x1, y1, x2, y2):
    """UpdatePushCharacterVsCharacter (BC:483-501) for two fighters on the base pushbox (Rect:
    x = position.x, y = position.y, width 1.4, height 1; Overlaps strict in x and y), float32,
    with the y carried as the C# passes it."""
    r1 = (x1, y1, F32(PUSH_W + x1), F32(PUSH_H + y1))  # (xMin, yMin, xMax = width + x, yMax)
    r2 = (x2, y2, F32(PUSH_W + x2), F32(PUSH_H + y2))
    if not (r2[2] > r1[0] and r2[0] < r1[2] and r2[3] > r1[1] and r2[1] < r1[3]):
        return x1, y1, x2, y2
    if x1 < x2:
        d = F32(r1[2] - r2[0])
        x1, y1 = F32(x1 + F32(F32(d * -1) / 2)), F32(y1 + y1)
        x2, y2 = F32(x2 + F32(F32(d * 1) / 2)), F32(y2 + y2)
    elif x1 > x2:
        d = F32(r2[2] - r1[0])
        x1, y1 = F32(x1 + F32(F32(d * 1) / 2)), F32(y1 + y1)
        x2, y2 = F32(x2 + F32(F32(d * -1) / 2)), F32(y2 + y1)  # fighter1's y, already shifted
    return x1, y1, x2, y2


def _push_stage(x, y):
    """UpdatePushCharacterVsBackground (BC:503-519): BoxBase x is the centre (xMin = x - w/2)."""
    half = F32(PUSH_W / 2)
    xmin, xmax = F32(x - half), F32(x + half)
    if xmin < -STAGE:
        return F32(x + F32(-STAGE - xmin)), F32(y + y)
    if xmax > STAGE:
        return F32(x + F32(STAGE - xmax)), F32(y + y)
    return x, y


def _expect_standing(backend, x1, y1, x2, y2, ticks):
    """Both fighters STAND without input for `ticks` ticks: only the pushes move them."""
    for t in range(ticks):
        x1, y1, x2, y2 = _push_pair(x1, y1, x2, y2)
        x1, y1 = _push_stage(x1, y1)
        x2, y2 = _push_stage(x2, y2)
        backend.step(_a(0), _a(0))
        f = backend.state()[0]["f"]
        got = (f[0]["position_x"], f[0]["position_y"], f[1]["position_x"], f[1]["position_y"])
        assert got == (x1, y1, x2, y2), (t, got, (x1, y1, x2, y2))
    return x1, y1, x2, y2


def kat_airborne_not_pushed(backend):
    """P1 at y = 2 over P2: the pushboxes overlap in x ([0, 1.4] and [0.5, 1.9]) but not in y
    ([2, 3] and [0, 1]), so neither moves and y stays 2; on the ground the same positions are
    pushed apart by 0.45 each (d = 1.4 - 0.5)."""
    fresh(backend)
    load_geom(backend, {"x": 0.0, "y": 2.0}, {"x": 0.5})
    _expect_standing(backend, F32(0.0), F32(2.0), F32(0.5), F32(0.0), 3)
    fresh(backend)
    load_geom(backend, {"x": 0.0}, {"x": 0.5})
    x1, _, x2, _ = _expect_standing(backend, F32(0.0), F32(0.0), F32(0.5), F32(0.0), 1)
    assert x1 < F32(0.0) < F32(0.5) < x2


def kat_stage_push_doubles_y(backend):
    """P1 loaded at x = -5.5, y = 0.25: its pushbox ([-6.2, -4.8]) is past the stage edge, so the
    background push moves it in by 1.2 and ApplyPositionChange(dx, position.y) doubles its y to
    0.5; back inside, it is not pushed again and y stays 0.5."""
    fresh(backend)
    load_geom(backend, {"x": -5.5, "y": 0.25}, {"x": 2.0})
    x1, y1, _, _ = _expect_standing(backend, F32(-5.5), F32(0.25), F32(2.0), F32(0.0), 3)
    assert y1 == F32(0.5) and x1 > F32(-5.5)


def kat_character_push_carries_y(backend):
    """Both at y = 0.25 with overlapping pushboxes.  P1 on the left: each is pushed by half the
    overlap and each y doubles (0.5, 0.5).  P1 on the right: P1's y doubles to 0.5 first, and
    P2 is shifted by P1's new y: 0.25 + 0.5 = 0.75 (BC:496-497 pass fighter1.position.y)."""
    fresh(backend)
    load_geom(backend, {"x": 0.0, "y": 0.25}, {"x": 0.5, "y": 0.25})
    _, y1, _, y2 = _expect_standing(backend, F32(0.0), F32(0.25), F32(0.5), F32(0.25), 3)
    assert (y1, y2) == (F32(0.5), F32(0.5))
    fresh(backend)
    load_geom(backend, {"x": 0.5, "y": 0.25}, {"x": 0.0, "y": 0.25})
    _, y1, _, y2 = _expect_standing(backend, F32(0.5), F32(0.25), F32(0.0), F32(0.25), 3)
    assert (y1, y2) == (F32(0.5), F32(0.75))


def _hit_expectation():
    a = ATTACKS[1]  # N_ATTACK's attack (ACT/N_ATTACK.asset: attackID 1)
    return a["guard_damage"], a["hit_stun"]


def kat_hit_needs_y_overlap(backend):
    """P2 in N_ATTACK frame 3 at x = 1 (facing left): on the next tick its real hitbox (frames
    4-5, rect x 0.9 w 1.8 h 0.3 -> x [-0.8, 1.0], y [0, 0.3]) overlaps P1's base hurtbox (x -0.5,
    w 1.5 -> [-1.25, 0.25]) in x.  In y the hurtbox is [y1, y1 + 1.2]: BoxBase.Overlaps is
    inclusive, so y1 = 0.3 (touching from above) and y1 = -1.2 (yMax = 0, touching from below)
    are hit -- DAMAGE, guard 3 -> 3 - guardDamage, hitstun = hitStun, reward -0.3 -- and 0.31 /
    -1.21 are not (STAND, guard 3, reward 0).  No push: the pushboxes [-0.5, 0.9] and [1, 2.4] do
    not overlap."""
    hb = [h for h in ACTIONS[N_ATTACK]["hitboxes"] if not h["proximity"]][0]
    assert hb["win"] == [4, 5] and hb["rect"] == [0.9, 0.0, 1.8, 0.3]
    gd, stun = _hit_expectation()
    for y1, hit in ((0.3, True), (0.31, False), (-1.2, True), (-1.21, False), (0.0, True)):
        fresh(backend)
        load_geom(backend, {"x": -0.5, "y": y1}, {"x": 1.0, "act": N_ATTACK, "frame": 3})
        out = backend.step(_a(0), _a(0))
        s = backend.env_state()[0]
        assert s["p2Move"] == N_ATTACK and s["p2MoveFrame"] == 4
        assert (s["p1Move"] == DAMAGE) == hit, (y1, s["p1Move"])
        assert s["p1Guard"] == (3 - gd if hit else 3) and s["p1Hitstun"] == (stun if hit else 0), y1
        assert out["reward"][0] == (-0.3 if hit else 0.0), (y1, out["reward"][0])
        assert backend.state()[0]["f"][0]["position_y"] == F32(y1)  # no push moved it


def kat_flipped_attacker(backend):
    """P2 loaded facing right at x = -1 in N_ATTACK frame 3, P1 at x = 0.5: mirrored, P2's real
    hitbox on the next tick spans x -1 + 0.9 +- 0.9 = [-1.0, 0.8] and reaches P1's hurtbox
    [-0.25, 1.25]: DAMAGE.  Facing left (its own facing) the hitbox would span [-2.8, -1.0] and
    P1 is untouched."""
    gd, stun = _hit_expectation()
    for flip, hit in ((1, True), (0, False)):
        fresh(backend)
        load_geom(backend, {"x": 0.5}, {"x": -1.0, "act": N_ATTACK, "frame": 3, "flip": flip})
        out = backend.step(_a(0), _a(0))
        s = backend.env_state()[0]
        assert (s["p1Move"] == DAMAGE) == hit and s["p1Guard"] == (3 - gd if hit else 3), (flip, s["p1Move"])
        assert out["reward"][0] == (-0.3 if hit else 0.0)
        assert s["p1Position"] == F32(0.5) and s["p2Position"] == F32(-1.0)


def kat_round_start_restores_geometry(backend):
    """The round start puts both fighters back on the ground facing each other: SetupBattleStart
    sets position = (+-2, 0) and isFaceRight = isPlayerOne (F:120-135, BC:264-265).  P1 is loaded
    flipped at y = 0.3 with vitalHealth 0, so the tick ends in KO (BC:212-213) and the same-step
    auto-reset runs the round start: the arena is standard again."""
    fresh(backend)
    load_geom(backend, {"x": -0.5, "y": 0.3, "flip": 1}, {"x": 1.0, "y": -0.7, "flip": 1})
    s = backend.state()
    s["f"][0, 0]["vital"] = 0
    backend.set_state(s)
    out = backend.step(_a(0), _a(0))
    assert out["terminated"][0] == 1
    f = backend.state()[0]["f"]
    assert (f[0]["position_y"], f[1]["position_y"]) == (0, 0) and (f[0]["facing_flipped"], f[1]["facing_flipped"]) == (0, 0)
    assert (f[0]["position_x"], f[1]["position_x"]) == (F32(_DATA["stage"]["p1_start_x"]),
                                                        F32(_DATA["stage"]["p2_start_x"]))


def kat_negative_zero_y(backend):
    """position.y loaded as -0.0 (STATE_LOAD, F:741-744) is kept bit for bit while the fighter
    stands and is pushed (each push adds y to itself: -0.0 + -0.0 = -0.0, BC:491-498, 511-515),
    and the round start writes +0.0 (SetupBattleStart's new Vector2(-2f, 0f), BC:264-265, F:120-135).
    P1 stands past the stage edge (x -5.5: pushed in, y doubled), then is loaded with vital 0 so
    the next tick ends the round and the same-step auto-reset runs the round start."""
    fresh(backend)
    load_geom(backend, {"x": -5.5, "y": -0.0}, {"x": 2.0, "y": -0.0})
    f = backend.state()[0]["f"]
    assert np.signbit(f[0]["position_y"]) and np.signbit(f[1]["position_y"])
    x1, y1, _, y2 = _expect_standing(backend, F32(-5.5), F32(-0.0), F32(2.0), F32(-0.0), 3)
    f = backend.state()[0]["f"]
    assert x1 > F32(-5.5) and np.signbit(f[0]["position_y"]) and np.signbit(f[1]["position_y"])
    s = backend.state()
    s["f"][0, 0]["vital"] = 0
    backend.set_state(s)
    assert backend.step(_a(0), _a(0))["terminated"][0] == 1
    f = backend.state()[0]["f"]
    assert not np.signbit(f[0]["position_y"]) and not np.signbit(f[1]["position_y"])
    assert f[0]["position_y"] == 0 and f[1]["position_y"] == 0


ALL = {
    "negative_zero_y": kat_negative_zero_y,
    "flipped_walk": kat_flipped_walk,
    "airborne_not_pushed": kat_airborne_not_pushed,
    "stage_push_doubles_y": kat_stage_push_doubles_y,
    "character_push_carries_y": kat_character_push_carries_y,
    "hit_needs_y_overlap": kat_hit_needs_y_overlap,
    "flipped_attacker": kat_flipped_attacker,
    "round_start_restores_geometry": kat_round_start_restores_geometry,
}
