"""BattleState save / load in the reference's JSON format (STATE_SAVE / STATE_LOAD).

Reference: BattleCore.SaveState / LoadState (BattleCore.cs:667-683), BattleState.cs:7-24,
FighterState.cs:9-133, Fighter.SaveState / LoadState (Fighter.cs:721-811), and the Python
mirror FootsiesBattleState / FootsiesFighterState (footsies_gym/state.py:78-137).

The simulator's canonical per-arena state (fs_arena_state, include/footsies.h) holds
what the simulation reads.  The mapping is exact for every field a loaded state is
read through -- position, vital / guard health, action id / frame / hit count, hitstun,
buffer / reserve action, the two guard latches, hasWon, frameCount, the directions of
input[0..15] and the Attack bit over the held run input[0..hold-1] (hold saturating at
63) -- which covers every history read of the tick (dash parsers: input[0..16] after
the shift; charge special: input[1..59]).  The rest is rebuilt canonically on save and
ignored on load, because the simulation overwrites or never reads it:
  * hitboxes / hurtboxes / pushbox: recomputed by UpdateBoxes before any use
    (Fighter.cs:321-324, 671-697); saved as the current (action, frame) boxes at the
    current position;
  * velocity_x: assigned before being read in UpdateMovement (Fighter.cs:313-318);
    saved as the current frame's movement velocity (0 outside movement windows);
  * input / inputDown / inputUp beyond what is listed above: saved as zeros;
    inputDown / inputUp are derived from input (Fighter.cs:182-184);
  * spriteShakePosition / maxSpriteShakeFrame: rendering only (BattleGUI.cs:128, 139);
    saved as 0 / 6 (Fighter.cs:110);
  * roundStartTime: only stamps recorded inputs (BattleCore.cs:390, 420); saved as 0.
Fields outside BattleState (bot RNG and queues, recording index, FootsiesEnv reward
accumulator) keep the arena's current values on load, as STATE_LOAD leaves them.
"""
import dataclasses
import json
import os
from typing import List

import numpy as np

from . import _abi
from ._lib import FootsiesError

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INPUT_RECORD_FRAME = 180  # Fighter.inputRecordFrame (Fighter.cs:98-101)
MAX_SPRITE_SHAKE_FRAME = 6  # Fighter.cs:110
IN_LEFT, IN_RIGHT, IN_ATTACK = 1, 2, 4  # InputData.cs:8-14

_FRAME_DATA = {}


def frame_data():
    """The F00 frame data extracted from the reference assets (data/f00.json, tools/extract_f00.py)."""
    if "d" not in _FRAME_DATA:
        with open(os.path.join(ROOT, "data", "f00.json")) as f:
            d = json.load(f)
        d["by_id"] = {a["id"]: a for a in d["actions"]}
        _FRAME_DATA["d"] = d
    return _FRAME_DATA["d"]


def _in_window(win, frame):
    return win[0] <= frame <= win[1]


def _world_rect(rect, x, y, sign):
    """TransformToFightRect (Fighter.cs:700-715), float32 arithmetic."""
    f32 = np.float32
    return {"x": float(f32(f32(x) + f32(f32(rect[0]) * f32(sign)))), "y": float(f32(f32(y) + f32(rect[1]))),
            "width": float(f32(rect[2])), "height": float(f32(rect[3]))}


def _boxes(action_id, frame, x, y, face_right):
    """ApplyCurrentActionData (Fighter.cs:671-697) for (action, frame) at position (x, y)."""
    d = frame_data()
    a = d["by_id"][action_id]
    sign = 1 if face_right else -1
    base_hurt, base_push = d["fighter"]["base_hurtbox"], d["fighter"]["base_pushbox"]
    hit = [{"rect": _world_rect(h["rect"], x, y, sign), "proximity": bool(h["proximity"]),
            "attackID": int(h["attack_id"])} for h in a["hitboxes"] if _in_window(h["win"], frame)]
    hurt = [_world_rect(base_hurt if h["use_base"] else h["rect"], x, y, sign)
            for h in a["hurtboxes"] if _in_window(h["win"], frame)]
    push = next((p for p in a["pushboxes"] if _in_window(p["win"], frame)), None)
    push_rect = base_push if push is None or push["use_base"] else push["rect"]
    velocity = next((m["velocity_x"] for m in a["movements"] if _in_window(m["win"], frame)), 0.0)
    return hit, hurt, _world_rect(push_rect, x, y, sign), float(np.float32(velocity))


def _input_arrays(dir_history, hold):
    """input / inputDown / inputUp (Fighter.cs:172-188) from the canonical history."""
    inp = np.zeros(INPUT_RECORD_FRAME + 1, dtype=np.int64)  # one spare zero past the end
    for j in range(16):
        inp[j] = (int(dir_history) >> (2 * j)) & 3
    inp[:min(int(hold), INPUT_RECORD_FRAME)] |= IN_ATTACK
    changed = inp[:-1] ^ inp[1:]
    down = changed & inp[:-1]
    up = changed & ~inp[:-1]
    return [int(v) for v in inp[:-1]], [int(v) for v in down], [int(v) for v in up]


def fighter_state(f, is_p1):
    """One fs_fighter_state record -> FighterState dict (FighterState.cs field order)."""
    x = float(np.float32(f["position_x"]))
    y = float(np.float32(f["position_y"]))
    face_right = bool(is_p1) != bool(f["facing_flipped"])  # SetupBattleStart: isFaceRight = isPlayerOne
    act = int(f["action_id"])
    hit, hurt, push, vel = _boxes(act, int(f["action_frame"]), x, y, face_right)
    inp, down, up = _input_arrays(f["input_dir_history"], f["attack_hold"])
    return {
        "position": [x, y], "velocity_x": vel, "isFaceRight": face_right,
        "hitboxes": hit, "hurtboxes": hurt, "pushbox": push,
        "vitalHealth": int(f["vital"]), "guardHealth": int(f["guard"]),
        "currentActionID": act, "currentActionFrame": int(f["action_frame"]),
        "currentActionHitCount": int(f["hit_count"]), "currentHitStunFrame": int(f["hitstun"]),
        "input": inp, "inputDown": down, "inputUp": up,
        "isInputBackward": bool(f["is_input_backward"]), "isReserveProximityGuard": bool(f["is_reserve_proximity_guard"]),
        "bufferActionID": int(f["buffer_action_id"]), "reserveDamageActionID": int(f["reserve_action_id"]),
        "spriteShakePosition": 0, "maxSpriteShakeFrame": MAX_SPRITE_SHAKE_FRAME, "hasWon": bool(f["has_won"]),
    }


def battle_state(states, i):
    """Arena i of an fs_arena_state array -> BattleState dict (BattleState.cs:11-14 order)."""
    a = states[i]
    return {"p1State": fighter_state(a["f"][0], True), "p2State": fighter_state(a["f"][1], False),
            "roundStartTime": 0.0, "frameCount": int(a["frame_count"])}


def _float_text(v):
    """Floats as the shortest text that reads back as the same float32 (how Unity writes them)."""
    return repr(float(str(np.float32(v))))


def dumps(state):
    """JSON text of a BattleState dict; floats in shortest float32 round-trip form."""
    def enc(o):
        if isinstance(o, bool):
            return "true" if o else "false"
        if isinstance(o, float):
            return _float_text(o)
        if isinstance(o, int):
            return str(o)
        if isinstance(o, list):
            return "[" + ",".join(enc(v) for v in o) + "]"
        if isinstance(o, dict):
            return "{" + ",".join(json.dumps(k) + ":" + enc(v) for k, v in o.items()) + "}"
        raise TypeError(type(o))
    return enc(state)


class UnsupportedBattleStateError(FootsiesError, ValueError):
    """A BattleState the simulator cannot represent (a position that is not [x, y]).  Since round
    4 position.y != 0 and a flipped isFaceRight are loaded as Fighter.LoadState restores them
    (Fighter.cs:741-744) and run on the kernels' general-geometry tick (fs_set_state)."""

    def __init__(self, message):
        FootsiesError.__init__(self, _abi.FS_E_UNSUPPORTED, message)


def _load_fighter(dst, s, is_p1):
    """Fighter.LoadState (Fighter.cs:741-811) onto one fs_fighter_state record: position (x, y)
    and isFaceRight as given (a y other than 0 or a facing other than the player's own runs on
    the general-geometry tick, fs_set_state).  Raises UnsupportedBattleStateError for a position
    that is not [x, y]."""
    who = "p1State" if is_p1 else "p2State"
    pos = list(s["position"])
    if len(pos) != 2:
        raise UnsupportedBattleStateError("%s.position must be [x, y], got %r" % (who, pos))
    dst["position_x"] = np.float32(pos[0])
    dst["position_y"] = np.float32(pos[1])
    dst["facing_flipped"] = int(bool(s["isFaceRight"]) != bool(is_p1))
    dst["action_id"] = int(s["currentActionID"])
    dst["action_frame"] = int(s["currentActionFrame"])
    dst["hit_count"] = int(s["currentActionHitCount"])
    dst["hitstun"] = int(s["currentHitStunFrame"])
    dst["vital"] = int(s["vitalHealth"])
    dst["guard"] = int(s["guardHealth"])
    dst["buffer_action_id"] = int(s["bufferActionID"])
    dst["reserve_action_id"] = int(s["reserveDamageActionID"])
    inp = list(s["input"]) + [0] * 16
    dirs = 0
    for j in range(16):
        dirs |= (int(inp[j]) & 3) << (2 * j)
    dst["input_dir_history"] = dirs
    hold = 0
    while hold < 63 and hold < len(s["input"]) and int(s["input"][hold]) & IN_ATTACK:
        hold += 1
    dst["attack_hold"] = hold
    dst["is_input_backward"] = int(bool(s["isInputBackward"]))
    dst["is_reserve_proximity_guard"] = int(bool(s["isReserveProximityGuard"]))
    dst["has_won"] = int(bool(s["hasWon"]))


def load_into(states, i, state):
    """BattleCore.LoadState (BattleCore.cs:676-683) onto arena i of an fs_arena_state array,
    in place: the BattleState fields are replaced, everything else is kept.  `state` is a
    BattleState dict or its JSON text."""
    if isinstance(state, str):
        state = json.loads(state)
    _load_fighter(states[i]["f"][0], state["p1State"], True)
    _load_fighter(states[i]["f"][1], state["p2State"], False)
    states["frame_count"][i] = int(state["frameCount"])
    return states


@dataclasses.dataclass
class FootsiesFighterState:
    """One fighter of a BattleState, with the field names of FighterState.cs:33-56."""
    position: List[float]
    velocity_x: float
    isFaceRight: bool
    hitboxes: List[dict]
    hurtboxes: List[dict]
    pushbox: dict
    vitalHealth: int
    guardHealth: int
    currentActionID: int
    currentActionFrame: int
    currentActionHitCount: int
    currentHitStunFrame: int
    input: List[int]
    inputDown: List[int]
    inputUp: List[int]
    isInputBackward: bool
    isReserveProximityGuard: bool
    bufferActionID: int
    reserveDamageActionID: int
    spriteShakePosition: int
    maxSpriteShakeFrame: int
    hasWon: bool


@dataclasses.dataclass
class FootsiesBattleState:
    """A whole BattleState (BattleState.cs:11-14) as the reference's Python client holds it."""
    p1State: FootsiesFighterState
    p2State: FootsiesFighterState
    roundStartTime: float
    frameCount: int

    @staticmethod
    def from_dict(d):
        return FootsiesBattleState(FootsiesFighterState(**d["p1State"]), FootsiesFighterState(**d["p2State"]),
                                   float(d["roundStartTime"]), int(d["frameCount"]))

    @staticmethod
    def from_json(text):
        return FootsiesBattleState.from_dict(json.loads(text))

    def to_dict(self):
        return dataclasses.asdict(self)

    def json(self):
        return dumps(self.to_dict())
