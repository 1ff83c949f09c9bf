"""Replays of tests/golden/wrapper_golden.npz (made by tests/golden/make_wrapper_golden.py
from the reference's own wrappers) on any base vector env with reset / step / step_masked."""
import os

import numpy as np

from footsies_gym_amd import wrappers as W

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = ("skip_norm", "skip_raw", "norm_noguard", "stats_disc", "skip_delay")
STACKS = {
    "skip_norm": lambda b: W.FootsiesFrameSkipped(W.FootsiesNormalized(b, exact=True)),
    "skip_raw": lambda b: W.FootsiesFrameSkipped(b),
    "norm_noguard": lambda b: W.FootsiesNormalized(b, normalize_guard=False, exact=True),
    "stats_disc": lambda b: W.FootsiesStatistics(W.FootsiesActionCombinationsDiscretized(b)),
    "skip_delay": lambda b: W.FootsiesFrameSkipped(b),
}
_CACHE = {}


def load():
    if "z" not in _CACHE:
        with np.load(os.path.join(HERE, "golden", "wrapper_golden.npz")) as z:
            _CACHE["z"] = {k: z[k] for k in z.files}
    return _CACHE["z"]


def _check_obs(name, obs, exp, t):
    for k in ("guard", "move", "move_frame", "position"):
        got = np.asarray(obs[k])
        want = exp(k)
        got = got.reshape(want.shape)
        if got.dtype == np.float32:  # raw float32 obs: FE's value is the float32's decimal text
            assert np.array_equal(got.view(np.uint32), want.astype(np.float32).view(np.uint32)), (name, k, t)
        else:
            assert np.array_equal(got.astype(np.float64).view(np.uint64), want.view(np.uint64)), (name, k, t)


def replay(name, make_base):
    """make_base(n, dense, seed, frame_delay) -> a next_step-autoreset vector env with the bot
    as P2."""
    z = load()
    n, steps, seed, dense = (int(v) for v in z[name + "/config"])
    delay = int(z.get(name + "/frame_delay", 0))
    env = STACKS[name](make_base(n, bool(dense), seed, delay))
    obs, _ = env.reset()
    _check_obs(name, obs, lambda k: z["%s/first/%s" % (name, k)], -1)
    acts = z[name + "/actions"]
    for t in range(steps):
        a = acts[t].astype(np.int64) if name == "stats_disc" else W.FootsiesActionCombinationsDiscretized.action(acts[t])
        obs, rew, term, trunc, _ = env.step(a)
        _check_obs(name, obs, lambda k: z["%s/%s" % (name, k)][t], t)
        assert np.array_equal(np.asarray(rew, np.float64).view(np.uint64),
                              z[name + "/reward"][t].view(np.uint64)), (name, "reward", t)
        assert np.array_equal(np.asarray(term).astype(np.uint8), z[name + "/terminated"][t]), (name, "term", t)
        assert not np.asarray(trunc).any()
    if name == "stats_disc":
        for i in range(n):
            assert env.metric_special_moves_per_episode[i] == list(z["%s/stats/%d" % (name, i)]), i
            assert env.metric_special_moves_from_neutral_per_episode[i] == list(
                z["%s/stats_neutral/%d" % (name, i)]), i
        rep = env.report()
        assert rep["episodes"] == int(z[name + "/terminated"].sum())
    env.close()
