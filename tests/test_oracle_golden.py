"""The CPU oracle against golden vectors produced by the reference's own FootsiesEnv
(obs, info, reward, termination, reset handshake).  See tests/golden/make_golden.py."""
import pytest

from tests import golden_utils as gu


def oracle_backend(oracle_lib):
    def make(n, p2_mode, dense, autoreset, seed, frame_delay=0):
        o = oracle_lib.Oracle(n, p2_mode=p2_mode, dense_reward=dense, autoreset_mode=autoreset, base_seed=seed,
                              frame_delay=frame_delay)

        class B:
            def reset(self):
                return o.reset()

            def step(self, a1, a2):
                return o.step(a1, a2)
        return B()
    return make


@pytest.mark.parametrize("name", gu.CASES)
def test_oracle_matches_reference_fe_next_step(oracle_lib, name):
    gu.replay_next_step(gu.case(gu.load(), name), oracle_backend(oracle_lib))


@pytest.mark.parametrize("name", gu.CASES)
def test_oracle_matches_reference_fe_same_step(oracle_lib, name):
    gu.replay_same_step(gu.case(gu.load(), name), oracle_backend(oracle_lib))
