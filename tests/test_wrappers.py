"""Vectorized wrappers (footsies_gym_amd/wrappers.py) against golden vectors from the
reference's own wrappers (tests/golden/make_wrapper_golden.py), over the oracle-backed
test double on CPU; the GPU replay is in test_gpu_api.py."""
import numpy as np
import pytest

from footsies_gym_amd import wrappers as W
from tests import wrapper_replay as wr
from tests.oracle_vector_env import OracleVectorEnv


@pytest.mark.parametrize("name", wr.CASES)
def test_wrappers_match_reference_on_oracle(oracle_lib, name):
    wr.replay(name, lambda n, dense, seed, delay: OracleVectorEnv(n, oracle_lib, dense_reward=dense, seed=seed,
                                                                  frame_delay=delay))


def test_discretized_action_bits():
    a = W.FootsiesActionCombinationsDiscretized.action(np.arange(8))
    assert a.tolist() == [[bool(i & 1), bool(i & 2), bool(i & 4)] for i in range(8)]


def test_normalized_fast_path_close_to_exact(oracle_lib):
    base = OracleVectorEnv(64, oracle_lib, seed=3)
    fast = W.FootsiesNormalized(base)
    exact = W.FootsiesNormalized(base, exact=True)
    obs, _ = base.reset()
    rng = np.random.default_rng(0)
    for _ in range(200):
        obs, *_ = base.step(rng.integers(0, 8, 64))
        f, e = fast.observation(obs), exact.observation(obs)
        for k in ("guard", "position", "move_frame"):
            want = e[k].astype(np.float32)
            assert np.all(np.abs(f[k].view(np.int32).astype(np.int64) - want.view(np.int32)) <= 1), k
        undone = W.FootsiesNormalized.undo(e)
        assert np.allclose(undone["position"], obs["position"], rtol=0, atol=1e-6)


def test_normalized_must_wrap_base(oracle_lib):
    base = OracleVectorEnv(2, oracle_lib)
    with pytest.raises(ValueError):
        W.FootsiesNormalized(W.FootsiesStatistics(base))


def test_frame_skipped_space():
    from footsies_gym_amd import spaces as sp
    s = sp.frame_skipped_observation_space(sp.normalized_observation_space())
    assert s["move_frame"].shape == (1,) and float(s["move_frame"].high[0]) == 1.0
