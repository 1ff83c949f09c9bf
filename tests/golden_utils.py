"""Replays of tests/golden/fe_golden.npz (made by tests/golden/make_golden.py from the
reference's own FootsiesEnv) on any backend with the Oracle/FootsiesSim step interface."""
import os

import numpy as np

from footsies_gym_amd import _abi

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = ("bot_dense", "ext_dense", "bot_sparse", "ext_delay3", "bot_delay1", "ext_delay16")


_CACHE = {}


def load():
    """All arrays of the fixture, decompressed once (NpzFile re-reads on every access)."""
    if "g" not in _CACHE:
        with np.load(os.path.join(HERE, "golden", "fe_golden.npz")) as z:
            _CACHE["g"] = {k: z[k] for k in z.files}
    return _CACHE["g"]


def case(g, name):
    cfg = g[name + "/config"]
    return {"p2_mode": int(cfg[0]), "dense": bool(cfg[1]), "n": int(cfg[2]), "steps": int(cfg[3]),
            "seed": int(cfg[4]), "frame_delay": int(cfg[5]) if len(cfg) > 5 else 0, "g": g, "name": name}


def expected(c, key, t=None):
    a = c["g"]["%s/%s" % (c["name"], key)]
    return a if t is None else a[t]


def check_obs_row(c, out, t, rows, src_t=None, prefix="", first=False):
    """Compare outputs (rows `rows`) with the reference FE obs/info of fixture step src_t."""
    g = (lambda k: c["g"]["%s/first/%s" % (c["name"], k)]) if first else (lambda k: expected(c, k, src_t))
    assert np.array_equal(out[prefix + "guard"][rows].astype(np.int64), g("guard")[rows]), ("guard", t)
    assert np.array_equal(out[prefix + "move"][rows].astype(np.int64), g("move")[rows]), ("move", t)
    assert np.array_equal(out[prefix + "move_frame"][rows], g("move_frame")[rows].astype(np.float32)), ("mf", t)
    # FE positions are the JSON round trip of the float32; cast back they must be the same bits
    assert np.array_equal(out[prefix + "position"][rows].view(np.uint32),
                          g("position")[rows].astype(np.float32).view(np.uint32)), ("position", t)
    assert np.array_equal(out[prefix + "frame"][rows], g("frame")[rows]), ("frame", t)
    act = out[prefix + "action"][rows]
    for k, col in (("p1_action", 0), ("p2_action", 1)):
        bits = g(k)[rows]
        enc = bits[:, 0] * 1 + bits[:, 1] * 2 + bits[:, 2] * 4
        assert np.array_equal(act[:, col], enc.astype(np.uint8)), (k, t)
    assert np.array_equal(out[prefix + "hitstun"][rows, 0], g("p1_hitstun")[rows]), ("p1_hitstun", t)
    assert np.array_equal(out[prefix + "hitstun"][rows, 1], g("p2_hitstun")[rows]), ("p2_hitstun", t)


def replay_next_step(c, make_backend):
    """next_step auto-reset: the fixture's own step alignment (reset steps ignore actions)."""
    n = c["n"]
    be = make_backend(n, c["p2_mode"], c["dense"], _abi.FS_AUTORESET_NEXT_STEP, c["seed"], c["frame_delay"])
    out = be.reset()
    all_rows = np.arange(n)
    check_obs_row(c, out, -1, all_rows, first=True)
    ext = c["p2_mode"] == _abi.FS_P2_EXTERNAL
    for t in range(c["steps"]):
        out = be.step(expected(c, "p1", t), expected(c, "p2", t) if ext else None)
        check_obs_row(c, out, t, all_rows, src_t=t)
        is_reset = expected(c, "is_reset", t).astype(bool)
        # reward / termination on env steps are the reference's; reset steps report 0 / False
        assert np.array_equal(out["reward"][~is_reset].view(np.uint64),
                              expected(c, "reward", t)[~is_reset].view(np.uint64)), ("reward", t)
        assert np.array_equal(out["terminated"].astype(bool), expected(c, "terminated", t).astype(bool)), t
        assert not out["reward"][is_reset].any()


def replay_same_step(c, make_backend):
    """same_step auto-reset: a fixture reset step is folded into the terminal step before it
    (obs = the fixture's reset obs, final_* = the fixture's terminal obs); each arena skips
    the actions of its reset steps, so arenas advance on their own fixture clocks."""
    n = c["n"]
    ext = c["p2_mode"] == _abi.FS_P2_EXTERNAL
    is_reset = expected(c, "is_reset").astype(bool)
    # per arena, the fixture steps that are real env steps
    steps = [np.nonzero(~is_reset[:, i])[0] for i in range(n)]
    m = min(len(s) for s in steps)
    be = make_backend(n, c["p2_mode"], c["dense"], _abi.FS_AUTORESET_SAME_STEP, c["seed"], c["frame_delay"])
    be.reset()
    rows = np.arange(n)
    p1a, p2a = expected(c, "p1"), expected(c, "p2")
    for j in range(m):
        src = np.array([steps[i][j] for i in range(n)])
        out = be.step(p1a[src, rows], p2a[src, rows] if ext else None)
        term = expected(c, "terminated")[src, rows].astype(bool)
        assert np.array_equal(out["terminated"].astype(bool), term), j
        assert np.array_equal(out["reward"].view(np.uint64), expected(c, "reward")[src, rows].view(np.uint64)), j
        for i in range(n):
            r = np.array([i])
            if term[i]:
                check_obs_row(c, out, j, r, src_t=src[i], prefix="final_")
                check_obs_row(c, out, j, r, src_t=src[i] + 1)  # the reset step's obs
            else:
                check_obs_row(c, out, j, r, src_t=src[i])
