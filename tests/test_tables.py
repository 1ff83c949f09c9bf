"""Frame data: the committed JSON matches the reference's asset values,
and both generated headers are up to date with it."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load():
    with open(os.path.join(ROOT, "data", "f00.json")) as f:
        return json.load(f)


def test_generated_headers_up_to_date():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_tables.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_fighter_constants():  # F00.asset:14-31
    f = load()["fighter"]
    assert f["start_guard_health"] == 3
    assert f["dash_allow_frame"] == 9  # the asset overrides FighterData.cs:18's default 10
    assert f["special_attack_hold_frame"] == 60
    assert f["can_cancel_on_whiff"] is False
    assert f["base_hurtbox"] == [0.0, 0.0, 1.5, 1.2]
    assert f["base_pushbox"] == [0.0, 0.0, 1.4, 1.0]
    assert abs(f["forward_move_speed"] - 2.2) < 1e-9 and abs(f["backward_move_speed"] - 1.8) < 1e-9


def test_action_table():  # ACT/*.asset, SURVEY.md §3.4
    acts = {a["id"]: a for a in load()["actions"]}
    expect_frames = {0: 24, 1: 24, 2: 24, 10: 16, 11: 22, 100: 22, 105: 21, 110: 44, 115: 55, 200: 17, 301: 23,
                     305: 15, 306: 15, 310: 36, 350: 1, 500: 500, 510: 33}
    assert {k: v["frame_count"] for k, v in acts.items()} == expect_frames
    assert [k for k, v in acts.items() if v["always_cancelable"]] == [0, 1, 2, 350]
    assert acts[510]["is_loop"] and acts[510]["loop_from"] == 5
    assert [k for k, v in acts.items() if v["type"] == 3] == [301, 305, 306, 350]
    # B_SPECIAL's overlapping movement windows: first match wins (frame 10 -> 2)
    assert [m["win"] for m in acts[115]["movements"]] == [[0, 2], [0, 10], [10, 15], [16, 16]]
    # cancel lists decoded from the little-endian int32 blobs (6e000000 == 110)
    assert [c["action_ids"] for c in acts[100]["cancels"]] == [[110], [110]]
    assert [c["win"] for c in acts[105]["cancels"]] == [[1, 2], [3, 5]]
    # DASH_BACKWARD / B_SPECIAL invulnerable startup (no hurtbox window)
    assert acts[11]["hurtboxes"][0]["win"] == [4, 21]
    assert acts[115]["hurtboxes"][0]["win"] == [6, 54]


def test_attack_table():  # F00_AttackDataContainer.asset:14-54
    atk = {a["id"]: a for a in load()["attacks"]}
    assert atk[1]["damage_action"] == 200 and atk[1]["guard_action"] == 306 and atk[1]["hit_stun"] == 12
    assert atk[2]["guard_action"] == 305
    for i in (10, 11):
        assert atk[i]["damage_action"] == 500 and atk[i]["vital_damage"] == 1 and atk[i]["hit_stun"] == 0
        assert atk[i]["guard_stun"] == 15
    assert all(a["guard_damage"] == 1 and a["guard_break_stun"] == 30 and a["number_of_hit"] == 1
               for a in atk.values())


def test_move_table_matches_reference_python():
    """moves.py:12-42 as imported from the reference (tests/golden/moves_golden.json)."""
    from footsies_gym_amd import _abi
    with open(os.path.join(ROOT, "tests", "golden", "moves_golden.json")) as f:
        g = json.load(f)
    assert {int(k): v for k, v in g["id_to_index"].items()} == _abi.MOVE_ID_TO_INDEX
    assert [(m[0], m[1], m[2]) for m in g["moves"]] == list(_abi.MOVES)
    acts = {a["id"]: a["frame_count"] for a in load()["actions"]}
    assert all(acts[mid] == dur for _, mid, dur in _abi.MOVES)  # durations == asset frameCount


@pytest.mark.skipif(not os.path.isdir("/root/reference/Assets/Fighter/F00"),
                    reason="the reference assets exist only in the build container")
def test_f00_json_re_extracts_identically_from_the_reference_assets(tmp_path):
    """data/f00.json is what tools/extract_f00.py reads out of the reference's Unity assets
    (F00.asset, F00_AttackDataContainer.asset, Actions/*.asset, BattleScene.unity,
    TimeManager.asset): a fresh extraction is byte-identical to the committed file."""
    import subprocess
    import sys
    out = tmp_path / "f00.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "extract_f00.py"), str(out)],
                       capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, FOOTSIES_REF="/root/reference"))
    assert r.returncode == 0, r.stderr[-2000:]
    assert out.read_bytes() == open(os.path.join(ROOT, "data", "f00.json"), "rb").read()


def test_move_table_derives_from_the_frame_data():
    """footsies_gym_amd.moves (the reference's moves.py surface): ids and durations are the
    actions' own, and each attack's startup / active / recovery are the frames before, inside
    and after its non-proximity hitbox windows in data/f00.json."""
    import json
    import os
    from footsies_gym_amd.moves import FOOTSIES_MOVE_ID_TO_INDEX, FOOTSIES_MOVE_INDEX_TO_MOVE, FootsiesMove
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    acts = {a["name"]: a for a in json.load(open(os.path.join(root, "data", "f00.json")))["actions"]}
    assert len(FOOTSIES_MOVE_INDEX_TO_MOVE) == len(acts) == 17
    for i, m in enumerate(FOOTSIES_MOVE_INDEX_TO_MOVE):
        a = acts[m.name]
        hb = [h["win"] for h in a["hitboxes"] if not h["proximity"]]
        if hb:
            lo, hi = min(w[0] for w in hb), max(w[1] for w in hb)
            frames = (lo, hi - lo + 1, a["frame_count"] - hi - 1)
        else:
            frames = (0, 0, 0)
        v = m.value
        assert (v.id, v.duration, v.startup, v.active, v.recovery) == (a["id"], a["frame_count"], *frames), m.name
        assert FOOTSIES_MOVE_ID_TO_INDEX[v.id] == i
    assert FootsiesMove.N_SPECIAL.value.startup == 11


def test_move_phase_tests_match_reference_python():
    """FootsiesMove.in_startup / in_active / in_recovery (moves.py:30-38): every move, every frame
    0 .. duration + 1, against the reference's own answers (tests/golden/moves_golden.json)."""
    from footsies_gym_amd.moves import FootsiesMove
    with open(os.path.join(ROOT, "tests", "golden", "moves_golden.json")) as f:
        g = json.load(f)
    assert set(g["phases"]) == {m.name for m in FootsiesMove}
    for m in FootsiesMove:
        got = [int(m.in_startup(fr)) | (int(m.in_active(fr)) << 1) | (int(m.in_recovery(fr)) << 2)
               for fr in range(m.value.duration + 2)]
        assert got == g["phases"][m.name], m.name
