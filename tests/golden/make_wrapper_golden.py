#!/usr/bin/env python3
"""Golden vectors for the vectorized wrappers, from the REFERENCE's own wrappers
(footsies_gym/wrappers/*.py) over its own FootsiesEnv (build container only).

Each reference env gets its own one-arena CPU oracle as "the game": an action sent
by FootsiesEnv.step (FE:518-528) ticks that oracle when FootsiesEnv reads the next
state, and a read without an action is the reset read (FE:496-499), which finishes
the post-KO burst or, after a RESET command, restarts the round.  So every env
advances at its own pace, as under the reference's frame-skipping wrapper.  The
oracle's arena i is seeded like arena i of a vector env with base seed `seed`.

Recorded per agent step (one wrapper.step or, after a terminal step, wrapper.reset):
the action, the observation, reward, terminated, and at the end the statistics
wrapper's metric lists.  Output (committed): tests/golden/wrapper_golden.npz.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_PY = "/root/reference/footsies-gym"
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(HERE, "_gym_stub"))
sys.path.insert(0, REF_PY)

from footsies_gym.envs.footsies import FootsiesEnv  # noqa: E402
from footsies_gym.state import FootsiesState  # noqa: E402
from footsies_gym.wrappers import (FootsiesActionCombinationsDiscretized, FootsiesFrameSkipped,  # noqa: E402
                                   FootsiesNormalized, FootsiesStatistics)

from footsies_gym_amd import _abi  # noqa: E402
from oracle import binding  # noqa: E402
from tests.golden.make_golden import state_json  # noqa: E402


class GameEnv(FootsiesEnv):
    """The reference FootsiesEnv whose game is a private one-arena oracle."""

    def __init__(self, seed, dense_reward, frame_delay=0):
        super().__init__(skip_instancing=True, dense_reward=dense_reward, frame_delay=frame_delay)
        self.game = binding.Oracle(1, p2_mode=_abi.FS_P2_BOT, dense_reward=dense_reward,
                                   autoreset_mode=_abi.FS_AUTORESET_NEXT_STEP, base_seed=seed)
        self._p1 = None
        self._reset_cmd = False

    def _connect_to_game(self, retry_delay=0.5):
        self._connected = True

    def _send_action(self, action, is_opponent=False):
        assert not is_opponent
        self._p1 = sum(int(bool(b)) << i for i, b in enumerate(action))

    def _remote_control_send_command(self, command, value=""):
        assert command.name == "RESET", command
        self._reset_cmd = True

    def _receive_and_update_state(self):
        if self._p1 is not None:  # FootsiesEnv.step: the game ticks with the sent action
            self.game.step(np.array([self._p1], np.uint8))
            self._p1 = None
        else:  # FootsiesEnv.reset: RESET command, or the KO -> ... -> Fight burst
            self.game.reset(flags=_abi.FS_RESET_HARD if self._reset_cmd else _abi.FS_RESET_IF_NEEDED)
            self._reset_cmd = False
        self._current_state = FootsiesState(**json.loads(state_json(self.game.env_state()[0])))
        return self._current_state


def as_tuple(a):
    return ((a & 1) != 0, (a & 2) != 0, (a & 4) != 0)


def run(name, stack, n, steps, seed, sticky, dense, discrete, frame_delay=0):
    rng = np.random.default_rng(seed + 7)
    bases = [GameEnv(seed + i, dense, frame_delay) for i in range(n)]
    envs = [stack(b) for b in bases]
    rec = {"guard": [], "move": [], "move_frame": [], "position": []}
    acts = np.zeros((steps, n), np.uint8)
    rew = np.zeros((steps, n), np.float64)
    term = np.zeros((steps, n), np.uint8)
    is_reset = np.zeros((steps, n), np.uint8)
    first = [e.reset(seed=None, options=None)[0] for e in envs]
    pending = np.zeros(n, bool)
    a = rng.integers(0, 8, n)
    for t in range(steps):
        a = np.where(rng.random(n) < sticky, a, rng.integers(0, 8, n))
        acts[t] = a
        row = []
        for i, e in enumerate(envs):
            if pending[i]:
                obs, _ = e.reset(seed=None, options=None)
                is_reset[t, i] = 1
                pending[i] = False
            else:
                obs, r, d, tr, _ = e.step(int(a[i]) if discrete else as_tuple(int(a[i])))
                assert tr is False
                rew[t, i], term[t, i] = r, d
                pending[i] = d
            row.append(obs)
        for k in rec:
            rec[k].append([np.asarray(o[k], dtype=np.float64).reshape(-1) for o in row])
    out = {"%s/actions" % name: acts, "%s/reward" % name: rew, "%s/terminated" % name: term,
           "%s/is_reset" % name: is_reset, "%s/config" % name: np.array([n, steps, seed, int(dense)], np.int64)}
    if frame_delay:
        out["%s/frame_delay" % name] = np.array(frame_delay, np.int64)
    for k in rec:
        out["%s/%s" % (name, k)] = np.array(rec[k])
        out["%s/first/%s" % (name, k)] = np.array([np.asarray(o[k], np.float64).reshape(-1) for o in first])
    for i, e in enumerate(envs):
        w = e
        while not isinstance(w, FootsiesStatistics) and hasattr(w, "env"):
            w = w.env
        if isinstance(w, FootsiesStatistics):
            out["%s/stats/%d" % (name, i)] = np.array(w.metric_special_moves_per_episode, np.int64)
            out["%s/stats_neutral/%d" % (name, i)] = np.array(w.metric_special_moves_from_neutral_per_episode,
                                                               np.int64)
    print(name, "episodes:", int(term.sum()), "resets:", int(is_reset.sum()))
    return out


def main():
    data = {}
    data.update(run("skip_norm", lambda b: FootsiesFrameSkipped(FootsiesNormalized(b)), 12, 700, 20, 0.7, True,
                    False))
    data.update(run("skip_raw", lambda b: FootsiesFrameSkipped(b), 12, 700, 30, 0.5, False, False))
    data.update(run("norm_noguard", lambda b: FootsiesNormalized(b, normalize_guard=False), 8, 500, 40, 0.5, True,
                    False))
    # frame skipping over FootsiesEnv's delayed-frame queue (FE:126-131, 532-535): every env's
    # queue advances with its own steps
    data.update(run("skip_delay", lambda b: FootsiesFrameSkipped(b), 12, 700, 60, 0.6, True, False, frame_delay=3))
    data.update(run("stats_disc", lambda b: FootsiesStatistics(FootsiesActionCombinationsDiscretized(b)), 16, 4000,
                    50, 0.97, True, True))
    np.savez_compressed(os.path.join(HERE, "wrapper_golden.npz"), **data)
    print("wrote wrapper_golden.npz")


if __name__ == "__main__":
    main()
