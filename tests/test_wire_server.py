"""The wire-compatible game server (footsies_gym_amd/server.py) against traffic recorded
with the reference's own FootsiesEnv client (tests/golden/make_wire_golden.py), on the
oracle-backed test double; the GPU-backed replay is in test_gpu_api.py."""
import struct

import pytest

from footsies_gym_amd import server as S
from tests import wire_replay
from tests.oracle_server_backend import OracleBackend


@pytest.mark.parametrize("name", wire_replay.CASES)
def test_server_replays_reference_client_traffic(oracle_lib, name):
    assert wire_replay.replay(name, lambda p2_bot, seed: OracleBackend(oracle_lib, p2_bot, seed)) > 1000


def test_framing_and_action_bits():
    assert S.frame(b"abc") == struct.pack("!I", 3) + b"abc"
    assert [S.action_bits(bytes([a & 1, a & 2, a & 4])) for a in range(8)] == list(range(8))
    assert S.action_bits(bytes([0, 7, 0])) == 2  # any non-zero byte is pressed


def test_state_json_field_order():
    import numpy as np
    from footsies_gym_amd import _abi
    rec = np.zeros(1, dtype=np.ctypeslib.as_array((_abi.fs_env_state * 1)()).dtype)[0]
    rec["p1Position"] = np.float32(-2.0)
    rec["p2Position"] = np.float32(1.692)
    txt = S.env_state_json(rec)
    assert txt.startswith('{"p1Vital":0,"p2Vital":0,') and '"p2Position":1.692,' in txt
    assert list(__import__("json").loads(txt)) == list(S.ENV_STATE_FIELDS)
