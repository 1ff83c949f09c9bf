"""BattleState save / load (footsies_gym_amd/battle_state.py).

* The JSON schema is pinned by the reference's own client class (fixture made by
  tests/golden/make_battle_state_golden.py: our JSON parsed and re-written by
  footsies_gym/state.py FootsiesBattleState).
* The canonical state (fs_arena_state) is complete: the oracle keeps the reference's
  full 180-deep input histories, boxes and velocity, yet an oracle loaded from the
  canonical state -- or from its BattleState JSON -- continues exactly like the original.
"""
import json
import os

import numpy as np
import pytest

from footsies_gym_amd import _abi, battle_state as B
from tests.parity_utils import compare_outputs, compare_states

HERE = os.path.dirname(os.path.abspath(__file__))


def test_schema_matches_reference_client():
    with open(os.path.join(HERE, "golden", "battle_state_golden.json")) as f:
        cases = json.load(f)
    assert cases
    for c in cases:
        ours, ref = json.loads(c["ours"]), json.loads(c["reference"])
        assert ours == ref
        assert list(ours) == list(ref) and list(ours["p1State"]) == list(ref["p1State"])
        assert len(ours["p1State"]["input"]) == B.INPUT_RECORD_FRAME


def _run(o, rng, steps, acts=None):
    n = o.n
    out = []
    for t in range(steps):
        a1, a2 = (acts[t] if acts is not None else (rng.integers(0, 8, n).astype(np.uint8),
                                                      rng.integers(0, 8, n).astype(np.uint8)))
        out.append(({k: np.array(v, copy=True) for k, v in o.step(a1, a2).items()}, (a1, a2)))
    return out


def _sticky_actions(rng, n, steps):
    a1, a2 = rng.integers(0, 8, n), rng.integers(0, 8, n)
    seq = []
    for _ in range(steps):
        a1 = np.where(rng.random(n) < 0.9, a1, rng.integers(0, 8, n))
        a2 = np.where(rng.random(n) < 0.9, a2, rng.integers(0, 8, n))
        seq.append((a1.astype(np.uint8), a2.astype(np.uint8)))
    return seq


@pytest.mark.parametrize("autoreset", [_abi.FS_AUTORESET_SAME_STEP, _abi.FS_AUTORESET_NEXT_STEP])
@pytest.mark.parametrize("via_json", [False, True])
def test_loaded_state_continues_exactly(oracle_lib, autoreset, via_json):
    n = 256
    rng = np.random.default_rng(autoreset * 10 + via_json)
    a = oracle_lib.Oracle(n, p2_mode=_abi.FS_P2_EXTERNAL, autoreset_mode=autoreset, base_seed=5)
    for cut in (40, 333, 120):
        _run(a, rng, cut, _sticky_actions(rng, n, cut))
        snap = a.state()
        b = oracle_lib.Oracle(n, p2_mode=_abi.FS_P2_EXTERNAL, autoreset_mode=autoreset, base_seed=77)
        if via_json:
            base = snap.copy()
            base["f"]["action_id"] = 0  # BattleState fields must all come from the JSON
            base["f"]["input_dir_history"] = 0
            base["f"]["attack_hold"] = 0
            base["f"]["position_x"] = 0.0
            base["frame_count"] = 0
            for i in range(n):
                B.load_into(base, i, B.dumps(B.battle_state(snap, i)))
            compare_states(snap, base)
            assert b.set_state(base) == 0
        else:
            assert b.set_state(snap) == 0
        compare_states(snap, b.state())
        acts = _sticky_actions(rng, n, 400)
        ra, rb = _run(a, rng, 400, acts), _run(b, rng, 400, acts)
        for t, ((oa, _), (ob, _)) in enumerate(zip(ra, rb)):
            compare_outputs(oa, ob, step=t, same_step=autoreset == _abi.FS_AUTORESET_SAME_STEP)
        compare_states(a.state(), b.state())
        b.close()


def test_battle_state_objects_roundtrip(oracle_lib):
    o = oracle_lib.Oracle(8, p2_mode=_abi.FS_P2_EXTERNAL, base_seed=3)
    _run(o, np.random.default_rng(1), 90)
    st = o.state()
    for i in range(8):
        doc = B.dumps(B.battle_state(st, i))
        obj = B.FootsiesBattleState.from_json(doc)
        assert obj.p2State.isFaceRight is False and obj.p1State.isFaceRight is True
        assert obj.json() == doc
        assert obj.p1State.currentActionID == int(st["f"][i, 0]["action_id"])
