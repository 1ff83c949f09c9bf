"""footsies_gym_amd.utils: the reference's get_dict_obs_from_vector_obs (footsies_gym/utils.py:7-41)
over gymnasium's flattened Dict layout (one-hot blocks per MultiDiscrete element, raveled Boxes).
gymnasium is absent here, so the reference function itself cannot run: the layout is checked
against gymnasium's documented flatten of MultiDiscrete / Box / Dict, and the helper by round trips
through FootsiesNormalized's forward transform (normalization.py:31-42)."""
import numpy as np
import pytest

from footsies_gym_amd import spaces as sp
from footsies_gym_amd.utils import flat_size, flatten_obs, get_dict_obs_from_vector_obs, unflatten_obs
from footsies_gym_amd.wrappers import DURATION, GUARD_SCALE, POSITION_SCALE


def random_obs(rng, n=None):
    lead = () if n is None else (n,)
    move = rng.integers(0, len(sp.RELEVANT_MOVES), lead + (2,))
    return {
        "guard": rng.integers(0, 4, lead + (2,)),
        "move": move,
        "move_frame": np.floor(rng.random(lead + (2,)) * DURATION[move]).astype(np.float32),
        "position": (rng.random(lead + (2,)) * 9.2 - 4.6).astype(np.float32),
    }


def normalize(obs, guard=True):
    o = dict(obs)
    if guard:
        o["guard"] = obs["guard"] / GUARD_SCALE
    o["position"] = obs["position"] / POSITION_SCALE
    o["move_frame"] = obs["move_frame"] / DURATION[obs["move"]]
    return o


def test_flat_layout_is_gymnasiums():
    space = sp.single_observation_space()
    n = len(sp.RELEVANT_MOVES)
    assert flat_size(space) == 4 + 4 + n + n + 2 + 2
    obs = {"guard": np.array([1, 3]), "move": np.array([0, n - 1]),
           "move_frame": np.array([5.0, 7.0], np.float32), "position": np.array([-1.5, 2.25], np.float32)}
    f = flatten_obs(space, obs)
    want = np.concatenate([np.eye(4)[1], np.eye(4)[3], np.eye(n)[0], np.eye(n)[n - 1], [5.0, 7.0], [-1.5, 2.25]])
    assert np.array_equal(f, want)
    back = unflatten_obs(space, f)
    for k in obs:
        assert np.array_equal(back[k], obs[k]), k
    assert back["guard"].dtype == np.int64 and back["position"].dtype == np.float32


@pytest.mark.parametrize("guard", [True, False])
@pytest.mark.parametrize("n", [None, 257])
def test_round_trip_through_normalization_and_flattening(guard, n):
    rng = np.random.default_rng(7 + (n or 0))
    obs = random_obs(rng, n)
    space = sp.normalized_observation_space(guard)
    flat = flatten_obs(space, normalize(obs, guard))
    got = get_dict_obs_from_vector_obs(flat, flattened=True, unflattenend_observation_space=space,
                                       normalized=True, normalized_guard=guard)
    assert np.array_equal(np.asarray(got["move"]), obs["move"])
    assert np.allclose(np.asarray(got["guard"], np.float64), obs["guard"], atol=1e-6)
    assert np.allclose(got["position"], obs["position"], atol=1e-5)
    assert np.allclose(got["move_frame"], obs["move_frame"], atol=1e-4)


def test_dict_input_and_errors():
    rng = np.random.default_rng(3)
    obs = random_obs(rng)
    got = get_dict_obs_from_vector_obs(normalize(obs), flattened=False)
    assert np.allclose(got["position"], obs["position"], atol=1e-5)
    same = get_dict_obs_from_vector_obs(obs, flattened=False, normalized=False)
    assert same is obs
    with pytest.raises(ValueError, match="unflattened observation space"):
        get_dict_obs_from_vector_obs(np.zeros(10), flattened=True)
    with pytest.raises(ValueError, match="assumed to be a dictionary"):
        get_dict_obs_from_vector_obs(np.zeros(10), flattened=False)
    with pytest.raises(ValueError, match="does not match"):
        unflatten_obs(sp.single_observation_space(), np.zeros(5))


def test_footsies_state_matches_reference_python():
    """FootsiesState.from_battle_state and str() (state.py:7-76) against the reference class's own
    values for the 18 BattleStates of battle_state_golden.json (tests/golden/make_state_golden.py)."""
    import dataclasses
    import json
    import os
    from footsies_gym_amd.state import FootsiesBattleState, FootsiesState
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with open(os.path.join(here, "battle_state_golden.json")) as f:
        states = json.load(f)
    with open(os.path.join(here, "state_golden.json")) as f:
        want = json.load(f)
    assert len(want) == len(states) > 0
    for w in want:
        s = FootsiesState.from_battle_state(FootsiesBattleState.from_json(states[w["case"]]["ours"]))
        got = json.loads(json.dumps(dataclasses.asdict(s)))  # tuples -> lists, as the fixture holds them
        assert got == w["fields"], w["case"]
        assert str(s) == w["str"], w["case"]


def test_footsies_state_from_env_state_record():
    from footsies_gym_amd import _abi
    from footsies_gym_amd.state import FootsiesState
    rec = np.zeros(1, dtype=np.dtype(_abi.fs_env_state))[0]
    rec["p1Vital"], rec["p2Guard"], rec["p1Move"], rec["p2MoveFrame"] = 1, 2, 7, 12
    rec["p1Position"], rec["globalFrame"], rec["p1MostRecentAction"], rec["p2MostRecentAction"] = -1.25, 99, 5, 2
    s = FootsiesState.from_env_state(rec)
    assert (s.p1Vital, s.p2Guard, s.p1Move, s.p2MoveFrame, s.globalFrame) == (1, 2, 7, 12, 99)
    assert s.p1Position == -1.25
    assert s.p1MostRecentAction == (True, False, True) and s.p2MostRecentAction == (False, True, False)
