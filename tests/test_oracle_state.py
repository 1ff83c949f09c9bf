"""The oracle's STATE_LOAD / STATE_SAVE on CPU: arbitrary canonical states (any action and
frame, buffers, reserves, latches, hasWon, bot queues mid-plan) load and save back unchanged
in every P2 mode, and stepping from them is deterministic."""
import numpy as np
import pytest

from footsies_gym_amd import _abi
from tests.parity_utils import random_states

P2 = {"external": _abi.FS_P2_EXTERNAL, "bot": _abi.FS_P2_BOT, "noop": _abi.FS_P2_NOOP}


@pytest.mark.parametrize("p2,p1_bot", [(p, False) for p in sorted(P2)] + [("external", True), ("bot", True)])
def test_oracle_state_roundtrip_and_determinism(oracle_lib, p2, p1_bot):
    n = 1024
    st = random_states(n, np.random.default_rng(5), p2=p2, p2_bot_frac=0.3)
    p1m = _abi.FS_P1_BOT if p1_bot else _abi.FS_P1_EXTERNAL
    a = oracle_lib.Oracle(n, p2_mode=P2[p2], base_seed=1, p1_mode=p1m)
    b = oracle_lib.Oracle(n, p2_mode=P2[p2], base_seed=2, p1_mode=p1m)
    assert a.set_state(st) == 0 and b.set_state(st) == 0
    back = a.state()
    for name in st.dtype.names:
        if name.startswith("pad"):
            continue
        if name == "f":
            for fn in st["f"].dtype.names:
                if not fn.startswith("pad"):
                    assert np.array_equal(st["f"][fn], back["f"][fn]), fn
        else:
            assert np.array_equal(st[name], back[name]), name
    rng = np.random.default_rng(6)
    for _ in range(50):
        p1 = rng.integers(0, 8, n).astype(np.uint8)
        q2 = rng.integers(0, 8, n).astype(np.uint8) if p2 == "external" else None
        oa, ob = a.step(p1, q2), b.step(p1, q2)
        for k in oa:
            assert np.array_equal(np.asarray(oa[k]), np.asarray(ob[k])), k
    assert a.state().tobytes() == b.state().tobytes()
