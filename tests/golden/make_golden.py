#!/usr/bin/env python3
"""Generate golden vectors from the REFERENCE's own Python (build container only).

What is pinned: the FootsiesEnv post-processing layer (footsies.py:336-405,
482-570): obs extraction, DEAD/WIN -> STAND substitution, move_frame
simplification, move-id -> index mapping, info, dense/sparse reward with its
float64 accumulation, termination, the reset handshake (no RESET after a
terminated episode) and the delayed-frame queue (frame_delay, FE:126-131, 493-504,
532-535; the game-side states do not depend on it, so the oracle feeding them runs
with frame_delay 0 and the reference FE applies its own queue).  The reference FootsiesEnv class is imported from
/root/reference with a throwaway `gymnasium` stub (tests/golden/_gym_stub) and
driven exactly as its socket would drive it: `_receive_and_update_state` is fed
Unity-style EnvironmentState JSON (JsonUtility field order, floats in shortest
round-trip form) produced by the CPU oracle; `_send_action`, `_connect_to_game`
and the remote-control requests are recorded instead of sent.

What is NOT pinned by this: the C# simulation that produces those states (no
Unity binary exists anywhere here) -- that is covered by hand-derived KATs
(tests/test_oracle_kat.py) and stays "parity unpinned" against Unity.

Outputs (committed): tests/golden/fe_golden.npz, tests/golden/moves_golden.json.
"""
import json
import os
import sys
from collections import deque

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_PY = "/root/reference/footsies-gym"
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(HERE, "_gym_stub"))
sys.path.insert(0, REF_PY)

import footsies_gym.moves as ref_moves  # noqa: E402
from footsies_gym.envs.footsies import FootsiesEnv  # noqa: E402

from footsies_gym_amd import _abi  # noqa: E402
from oracle import binding  # noqa: E402

FIELDS = ["p1Vital", "p2Vital", "p1Guard", "p2Guard", "p1Move", "p1MoveFrame", "p2Move", "p2MoveFrame",
          "p1Position", "p2Position", "globalFrame", "p1MostRecentAction", "p2MostRecentAction", "p1Hitstun",
          "p2Hitstun"]  # EnvironmentState.cs:12-26 declaration order (JsonUtility order)


def state_json(rec):
    parts = []
    for f in FIELDS:
        v = rec[f]
        if f.endswith("Position"):
            parts.append('"%s":%s' % (f, str(np.float32(v))))  # shortest round-trip float32 text
        else:
            parts.append('"%s":%d' % (f, int(v)))
    return "{" + ",".join(parts) + "}"


class FedEnv(FootsiesEnv):
    """The reference FootsiesEnv with its socket I/O replaced by a state queue."""

    def __init__(self, **kw):
        super().__init__(skip_instancing=True, **kw)
        self.feed = deque()
        self.sent = []
        self.commands = []

    def _connect_to_game(self, retry_delay=0.5):
        self._connected = True

    def _receive_and_update_state(self):
        from footsies_gym.state import FootsiesState
        self._current_state = FootsiesState(**json.loads(self.feed.popleft()))
        return self._current_state

    def _send_action(self, action, is_opponent=False):
        self.sent.append(tuple(action))

    def _remote_control_send_command(self, command, value=""):
        self.commands.append((command.name, value))


def obs_row(obs, info):
    return {
        "guard": np.array(obs["guard"], dtype=np.int64), "move": np.array(obs["move"], dtype=np.int64),
        "move_frame": np.array(obs["move_frame"], dtype=np.float64),
        "position": np.array(obs["position"], dtype=np.float64), "frame": info["frame"],
        "p1_action": np.array(info["p1_action"], dtype=bool), "p2_action": np.array(info["p2_action"], dtype=bool),
        "p1_hitstun": info["p1_hitstun"], "p2_hitstun": info["p2_hitstun"],
    }


def generate(name, p2_mode, dense, n, steps, seed, sticky, frame_delay=0):
    ora = binding.Oracle(n, p2_mode=p2_mode, dense_reward=dense, autoreset_mode=_abi.FS_AUTORESET_NEXT_STEP,
                         base_seed=seed)
    rng = np.random.default_rng(seed + 1000)
    envs = [FedEnv(dense_reward=dense, frame_delay=frame_delay) for _ in range(n)]
    st = ora.env_state()
    for i, e in enumerate(envs):
        e.feed.append(state_json(st[i]))
    first = [obs_row(*e.reset()) for e in envs]
    for e in envs:
        assert e.commands == [], e.commands  # has_terminated is True at construction: no RESET
    p1s = np.zeros((steps, n), np.uint8)
    p2s = np.zeros((steps, n), np.uint8)
    rows = []
    rew = np.zeros((steps, n), np.float64)
    term = np.zeros((steps, n), np.uint8)
    is_reset = np.zeros((steps, n), np.uint8)
    a1 = rng.integers(0, 8, n).astype(np.uint8)
    a2 = rng.integers(0, 8, n).astype(np.uint8)
    pending = np.zeros(n, bool)
    for t in range(steps):
        a1 = np.where(rng.random(n) < sticky, a1, rng.integers(0, 8, n)).astype(np.uint8)
        a2 = np.where(rng.random(n) < sticky, a2, rng.integers(0, 8, n)).astype(np.uint8)
        p1s[t], p2s[t] = a1, a2
        ora.step(a1, a2 if p2_mode == _abi.FS_P2_EXTERNAL else None)
        st = ora.env_state()
        out_t = []
        for i, e in enumerate(envs):
            e.feed.append(state_json(st[i]))
            if pending[i]:  # the agent calls reset() after a terminated step: FE reads state(-1)
                obs, info = e.reset()
                assert e.commands == [], e.commands
                is_reset[t, i] = 1
                pending[i] = False
            else:
                act = ((a1[i] & 1) != 0, (a1[i] & 2) != 0, (a1[i] & 4) != 0)
                obs, r, terminated, truncated, info = e.step(act)
                assert truncated is False
                rew[t, i] = r
                term[t, i] = terminated
                pending[i] = terminated
            out_t.append(obs_row(obs, info))
        rows.append(out_t)
    ora.close()

    def stack(key, src):
        return np.array([[r[key] for r in row] for row in src])

    out = {"%s/p1" % name: p1s, "%s/p2" % name: p2s, "%s/reward" % name: rew, "%s/terminated" % name: term,
           "%s/is_reset" % name: is_reset,
           "%s/config" % name: np.array([p2_mode, int(dense), n, steps, seed, frame_delay], dtype=np.int64)}
    for key in first[0]:
        out["%s/first/%s" % (name, key)] = np.array([r[key] for r in first])
        out["%s/%s" % (name, key)] = stack(key, rows)
    print(name, "episodes:", int(term.sum()), "resets:", int(is_reset.sum()))
    return out


def main():
    data = {}
    data.update(generate("bot_dense", _abi.FS_P2_BOT, True, 16, 2000, 0, 0.5))
    data.update(generate("ext_dense", _abi.FS_P2_EXTERNAL, True, 16, 1500, 1, 0.3))
    data.update(generate("bot_sparse", _abi.FS_P2_BOT, False, 16, 1500, 2, 0.8))
    data.update(generate("ext_delay3", _abi.FS_P2_EXTERNAL, True, 16, 1500, 3, 0.3, frame_delay=3))
    data.update(generate("bot_delay1", _abi.FS_P2_BOT, False, 16, 1200, 4, 0.6, frame_delay=1))
    data.update(generate("ext_delay16", _abi.FS_P2_EXTERNAL, True, 8, 800, 5, 0.5, frame_delay=16))
    np.savez_compressed(os.path.join(HERE, "fe_golden.npz"), **data)
    sys.path.insert(0, HERE)
    import make_moves_golden  # noqa: E402
    make_moves_golden.write(ref_moves)
    print("wrote fe_golden.npz, moves_golden.json")


if __name__ == "__main__":
    main()
