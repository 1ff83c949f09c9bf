#!/usr/bin/env python3
"""Extract the F00 frame-data assets of the reference into ``data/f00.json``.

Runs only in the build container (the GPU box never sees ``/root/reference``).
The output JSON is committed; everything downstream (the oracle's window
tables, the kernel's dense tables) is generated from it by
``tools/gen_tables.py``.

Sources (relative to the reference root):
  * fighter constants  Assets/Fighter/F00/F00.asset:14-31
  * attack table       Assets/Fighter/F00/F00_AttackDataContainer.asset:14-54
  * 17 actions         Assets/Fighter/F00/Actions/*.asset  (types: Assets/Script/ActionData.cs:7-85)
  * stage width        Assets/Scenes/BattleScene.unity:273 (BattleCore._battleAreaWidth)
  * fixed dt           ProjectSettings/TimeManager.asset:6 (Fixed Timestep)

Unity serialises ``List<int>`` (CancelData.actionID, ActionData.cs:57) as a
hex blob of little-endian int32s, e.g. ``6e000000`` == [110].
"""
import json
import os
import re
import struct
import sys

import yaml

REF = os.environ.get("FOOTSIES_REF", "/root/reference")
F00 = os.path.join(REF, "Assets/Fighter/F00")


def load_unity_yaml(path):
    lines = []
    with open(path, encoding="utf-8-sig") as f:
        for ln in f:
            if ln.startswith("%") or ln.startswith("---"):
                continue
            lines.append(ln)
    doc = yaml.safe_load("".join(lines))
    return doc["MonoBehaviour"]


def rect(r):
    return [float(r["x"]), float(r["y"]), float(r["width"]), float(r["height"])]


def int_list_blob(v):
    if v is None or v == "":
        return []
    if isinstance(v, int):  # yaml may parse an all-digit blob as int
        v = "%08d" % v
    v = str(v)
    assert len(v) % 8 == 0, v
    return [struct.unpack("<i", bytes.fromhex(v[i:i + 8]))[0] for i in range(0, len(v), 8)]


def window(d):
    se = d["startEndFrame"]
    return [int(se["x"]), int(se["y"])]


def parse_action(path):
    m = load_unity_yaml(path)
    act = {
        "id": int(m["actionID"]),
        "name": m["actionName"],
        "type": int(m["Type"]),
        "frame_count": int(m["frameCount"]),
        # isLoop / loopFromFrame / alwaysCancelable default to false/0 when omitted (ActionData.cs:75-84)
        "is_loop": bool(int(m.get("isLoop", 0) or 0)),
        "loop_from": int(m.get("loopFromFrame", 0) or 0),
        "always_cancelable": bool(int(m.get("alwaysCancelable", 0) or 0)),
        "hitboxes": [],
        "hurtboxes": [],
        "pushboxes": [],
        "movements": [],
        "cancels": [],
    }
    for h in m.get("hitboxes") or []:
        act["hitboxes"].append({"win": window(h), "rect": rect(h["rect"]),
                                "attack_id": int(h["attackID"]), "proximity": bool(int(h["proximity"]))})
    for h in m.get("hurtboxes") or []:
        act["hurtboxes"].append({"win": window(h), "rect": rect(h["rect"]),
                                 "use_base": bool(int(h["useBaseRect"]))})
    for h in m.get("pushboxes") or []:
        act["pushboxes"].append({"win": window(h), "rect": rect(h["rect"]),
                                 "use_base": bool(int(h["useBaseRect"]))})
    for h in m.get("movements") or []:
        act["movements"].append({"win": window(h), "velocity_x": float(h["velocity_x"])})
    for h in m.get("cancels") or []:
        act["cancels"].append({"win": window(h), "buffer": bool(int(h["buffer"])),
                               "execute": bool(int(h["execute"])),
                               "action_ids": int_list_blob(h.get("actionID"))})
    return act


def main(out_path):
    fd = load_unity_yaml(os.path.join(F00, "F00.asset"))
    fighter = {
        "start_guard_health": int(fd["startGuardHealth"]),
        "forward_move_speed": float(fd["forwardMoveSpeed"]),
        "backward_move_speed": float(fd["backwardMoveSpeed"]),
        "dash_allow_frame": int(fd["dashAllowFrame"]),
        "special_attack_hold_frame": int(fd["specialAttackHoldFrame"]),
        "can_cancel_on_whiff": bool(int(fd["canCancelOnWhiff"])),
        "base_hurtbox": rect(fd["baseHurtBoxRect"]),
        "base_pushbox": rect(fd["basePushBoxRect"]),
    }
    ad = load_unity_yaml(os.path.join(F00, "F00_AttackDataContainer.asset"))
    attacks = []
    for a in ad["attackDataList"]:
        attacks.append({
            "id": int(a["attackID"]), "name": a["attackName"],
            "damage_action": int(a["damageActionID"]), "guard_action": int(a["guardActionID"]),
            "number_of_hit": int(a["numberOfHit"]),
            "vital_damage": int(a["vitalHealthDamage"]), "guard_damage": int(a["guardHealthDamage"]),
            "hit_stun": int(a["hitStunFrame"]), "guard_stun": int(a["guardStunFrame"]),
            "guard_break_stun": int(a["guardBreakStunFrame"]),
        })
    acts_dir = os.path.join(F00, "Actions")
    actions = [parse_action(os.path.join(acts_dir, f)) for f in sorted(os.listdir(acts_dir)) if f.endswith(".asset")]
    actions.sort(key=lambda a: a["id"])

    scene = open(os.path.join(REF, "Assets/Scenes/BattleScene.unity"), encoding="utf-8").read()
    width = float(re.search(r"_battleAreaWidth:\s*([0-9.]+)", scene).group(1))
    tm = open(os.path.join(REF, "ProjectSettings/TimeManager.asset"), encoding="utf-8").read()
    dt = float(re.search(r"Fixed Timestep:\s*([0-9.]+)", tm).group(1))

    out = {
        "_source": "extracted by tools/extract_f00.py from the reference's F00 assets",
        "fighter": fighter,
        "attacks": attacks,
        "actions": actions,
        "stage": {"battle_area_width": width, "fixed_delta_time": dt,
                  "p1_start_x": -2.0, "p2_start_x": 2.0},  # BattleCore.cs:264-265
        "max_recording_input_frame": 60 * 60 * 5,        # BattleCore.cs:67
        "input_record_frame": 180,                        # Fighter.cs:98
    }
    with open(out_path, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print("wrote", out_path, len(actions), "actions", len(attacks), "attacks")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "data", "f00.json"))
