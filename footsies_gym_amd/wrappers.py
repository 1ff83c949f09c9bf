"""Vectorized counterparts of the reference's gymnasium wrappers (footsies_gym/wrappers/*.py).

Each wraps a FootsiesVectorEnv (numpy output) -- or another of these wrappers -- and
applies, per arena, what the reference wrapper does to one FootsiesEnv:

  FootsiesActionCombinationsDiscretized  action_comb_disc.py:6-18   int 0..7 -> (left, right, attack)
  FootsiesNormalized                     normalization.py:7-55      guard / 3, position / 4.6,
                                                                    move_frame / move duration
  FootsiesFrameSkipped                   frame_skip.py:6-80         no-op through frames where P1
                                                                    cannot act, summing rewards
  FootsiesStatistics                     statistics.py:5-70         special-move counts per episode

Auto-reset: the vector env resets finished arenas itself ("same_step" or
"next_step"); a "next_step" reset step reports state(-1) with reward 0, which
these wrappers treat like the reference wrapper's reset() (nothing is skipped or
counted on state(-1)).
"""
import numpy as np

from . import _abi
from . import spaces as sp

# move indices (FOOTSIES_MOVE_ID_TO_INDEX order, moves.py:41-42)
_IDX = {name: i for i, (name, _, _) in enumerate(_abi.MOVES)}
DURATION = np.array([d for _, _, d in _abi.MOVES], dtype=np.int64)  # FootsiesMove.value.duration
HIT_GUARD_MOVES = np.array([_IDX[m] for m in ("DAMAGE", "GUARD_STAND", "GUARD_CROUCH", "GUARD_M", "GUARD_BREAK")])
SPECIALS = np.array([_IDX["B_SPECIAL"], _IDX["N_SPECIAL"]])
NORMALS = np.array([_IDX["B_ATTACK"], _IDX["N_ATTACK"]])
POSITION_SCALE = 4.6  # normalization.py:36
GUARD_SCALE = 3.0     # normalization.py:35


class VectorWrapper:
    """Delegates everything it does not override to the wrapped vector env."""

    def __init__(self, env):
        self.env = env
        self.num_envs = env.num_envs

    def __getattr__(self, name):
        if name == "env":
            raise AttributeError(name)
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        e = self.env
        while isinstance(e, VectorWrapper):
            e = e.env
        return e

    def reset(self, *, seed=None, options=None):
        return self.env.reset(seed=seed, options=options)

    def step(self, actions):
        return self.env.step(actions)

    def step_masked(self, actions, active):
        return self.env.step_masked(actions, active)

    def close(self):
        return self.env.close()


def _map_final(info, fn):
    """Apply an observation transform to the same-step auto-reset terminal observations."""
    fo = info.get("final_observation")
    if fo is None:
        return info
    fo = fo.copy()
    for i in np.nonzero(info["_final_observation"])[0]:
        one = {k: np.asarray(v)[None] for k, v in fo[i].items()}
        fo[i] = {k: v[0] for k, v in fn(one).items()}
    info = dict(info)
    info["final_observation"] = fo
    return info


class FootsiesActionCombinationsDiscretized(VectorWrapper):
    """Actions are ints 0..7 per arena; bit 0 = left, bit 1 = right, bit 2 = attack -- the
    game's own input encoding (action_comb_disc.py:6-18, InputData.cs:8-14)."""

    def __init__(self, env):
        super().__init__(env)
        self.single_action_space = sp.Discrete(8)
        self.action_space = sp.MultiDiscrete(np.full(self.num_envs, 8))

    @staticmethod
    def action(act):
        a = np.asarray(act, dtype=np.int64).reshape(-1)
        return np.stack([(a & 1) != 0, (a & 2) != 0, (a & 4) != 0], axis=1)

    def step(self, actions):
        return self.env.step(self.action(actions))

    def step_masked(self, actions, active):
        return self.env.step_masked(self.action(actions), active)


def _decimal_f64(x):
    """float64 of the shortest decimal text of each float32 -- how EnvironmentState
    positions reach FootsiesEnv (JSON text parsed by Python, FE:319)."""
    x = np.asarray(x, dtype=np.float32)
    return np.array([float(s) for s in x.reshape(-1).astype(str)], dtype=np.float64).reshape(x.shape)


class FootsiesNormalized(VectorWrapper):
    """guard / 3 (optional), position / 4.6, move_frame / duration of the move, per arena
    (normalization.py:7-55).  Must wrap the base vector env, like the reference, which
    raises ValueError otherwise (normalization.py:18-19).

    ``exact=True`` reproduces the reference's float64 arithmetic bit for bit (positions are
    first turned into the decimal the JSON transport carries); the default path returns
    float32 within 1 ulp of float32(reference value) without per-element text conversion."""

    def __init__(self, env, normalize_guard=True, exact=False):
        if isinstance(env, VectorWrapper):
            raise ValueError("FootsiesNormalized should be applied to the base FOOTSIES vector environment")
        super().__init__(env)
        self.normalize_guard = normalize_guard
        self.exact = exact
        self.single_observation_space = sp.normalized_observation_space(normalize_guard)

    def observation(self, obs):
        o = dict(obs)
        move = np.asarray(obs["move"], dtype=np.int64)
        dur = DURATION[move]
        if self.exact:
            if self.normalize_guard:
                o["guard"] = np.asarray(obs["guard"], dtype=np.float64) / GUARD_SCALE
            o["position"] = _decimal_f64(obs["position"]) / POSITION_SCALE
            o["move_frame"] = np.asarray(obs["move_frame"], dtype=np.float64) / dur
        else:  # one rounding to float32 of the float64 quotient
            if self.normalize_guard:
                o["guard"] = (np.asarray(obs["guard"], dtype=np.float64) / GUARD_SCALE).astype(np.float32)
            o["position"] = (np.asarray(obs["position"], dtype=np.float64) / POSITION_SCALE).astype(np.float32)
            o["move_frame"] = (np.asarray(obs["move_frame"], dtype=np.float64) / dur).astype(np.float32)
        return o

    def reset(self, *, seed=None, options=None):
        obs, info = self.env.reset(seed=seed, options=options)
        return self.observation(obs), info

    def _wrap(self, res):
        obs, rew, term, trunc, info = res
        return self.observation(obs), rew, term, trunc, _map_final(info, self.observation)

    def step(self, actions):
        return self._wrap(self.env.step(actions))

    def step_masked(self, actions, active):
        return self._wrap(self.env.step_masked(actions, active))

    @staticmethod
    def undo(obs, normalized_guard=True):
        """Inverse transform (normalization.py:44-55)."""
        o = dict(obs)
        move = np.asarray(obs["move"], dtype=np.int64)
        if normalized_guard:
            o["guard"] = np.asarray(obs["guard"]) * GUARD_SCALE
        o["position"] = np.asarray(obs["position"]) * POSITION_SCALE
        o["move_frame"] = np.asarray(obs["move_frame"]) * DURATION[move]
        return o


def frame_skip_obs(obs):
    """P1's own move progress is dropped (frame_skip.py:40-47): move_frame keeps P2's only."""
    o = dict(obs)
    o["move_frame"] = np.asarray(obs["move_frame"])[:, 1:2]
    return o


def is_skippable(obs):
    """P1 is inside a move that has not (yet) hit or been blocked, or P1 is being hit
    (frame_skip.py:49-61)."""
    move = np.asarray(obs["move"])
    mf1 = np.asarray(obs["move_frame"])[:, 0]
    p2_hit_or_guarding = np.isin(move[:, 1], HIT_GUARD_MOVES)
    return ((mf1 != 0.0) & ~p2_hit_or_guarding) | (move[:, 0] == _IDX["DAMAGE"])


class FootsiesFrameSkipped(VectorWrapper):
    """Per arena, after the agent's action the arena keeps stepping with no input while
    its observation is skippable and the episode goes on; the rewards of those frames
    are summed into the step's reward (frame_skip.py:63-80).  Arenas advance at their
    own pace through fs_step_masked, so each one sees exactly the tick sequence of a
    separately wrapped FootsiesEnv.  Apply on top of FootsiesNormalized, not below it."""

    def __init__(self, env):
        super().__init__(env)
        self.single_observation_space = sp.frame_skipped_observation_space(env.single_observation_space)
        self._noop = np.zeros(self.num_envs, dtype=np.uint8)

    def reset(self, *, seed=None, options=None):
        obs, info = self.env.reset(seed=seed, options=options)
        return frame_skip_obs(obs), info  # no skipping on the first state (frame_skip.py:65-69)

    def step(self, actions):
        obs, rew, term, trunc, info = self.env.step(actions)
        obs = {k: np.array(v) for k, v in obs.items()}
        total = 0.0 + np.asarray(rew, dtype=np.float64)
        term, trunc = np.array(term), np.array(trunc)
        info = dict(info)
        pending = is_skippable(obs) & ~(term | trunc)
        while pending.any():
            o2, r2, t2, tr2, i2 = self.env.step_masked(self._noop, pending)
            total[pending] += np.asarray(r2)[pending]
            for k in obs:
                obs[k][pending] = np.asarray(o2[k])[pending]
            term[pending] = np.asarray(t2)[pending]
            trunc[pending] = np.asarray(tr2)[pending]
            for k, v in i2.items():
                if k in ("final_observation", "_final_observation", "final_info", "_final_info"):
                    continue
                info[k] = np.array(info[k])
                info[k][pending] = np.asarray(v)[pending]
            if "final_observation" in i2:
                _merge_final(info, i2, pending)
            pending &= is_skippable(obs) & ~(term | trunc)
        return frame_skip_obs(obs), total, term, trunc, _map_final(info, frame_skip_obs)


def _merge_final(info, new, rows):
    """Carry same-step auto-reset terminal entries of a masked step into the batch info."""
    n = len(rows)
    take = np.asarray(new["_final_observation"]) & rows
    if not take.any():
        return
    for key in ("final_observation", "final_info"):
        cur = info.get(key)
        if cur is None:
            cur = np.empty(n, dtype=object)
            info["_" + key] = np.zeros(n, dtype=bool)
        cur = cur.copy()
        cur[take] = new[key][take]
        info[key] = cur
        info["_" + key] = np.asarray(info["_" + key]) | take


class FootsiesStatistics(VectorWrapper):
    """Special-move counts per episode, per arena (statistics.py:5-70).  A special is
    counted when P1's move becomes N_SPECIAL or B_SPECIAL; "from neutral" when the move
    before it was not N_ATTACK / B_ATTACK.  As in the reference, only the first counter
    is recorded and cleared at each episode end (statistics.py:50-55): the from-neutral
    counter keeps accumulating and its per-episode list stays empty.  Wrap the base env
    (or FootsiesActionCombinationsDiscretized), below any observation wrapper."""

    def __init__(self, env):
        super().__init__(env)
        n = self.num_envs
        self._special = np.zeros(n, dtype=np.int64)
        self._special_neutral = np.zeros(n, dtype=np.int64)
        self._prev_move = np.full(n, -1, dtype=np.int64)
        self._per_episode = [[] for _ in range(n)]
        self._neutral_per_episode = [[] for _ in range(n)]

    def reset(self, *, seed=None, options=None):
        obs, info = self.env.reset(seed=seed, options=options)
        mask = None if not options or options.get("mask") is None else np.asarray(options["mask"], dtype=bool)
        move = np.asarray(obs["move"])[:, 0]
        if mask is None:
            self._prev_move[:] = move
        else:
            self._prev_move[mask] = move[mask]
        return obs, info

    def _count(self, obs, term, trunc, info, rows=None):
        move = np.asarray(obs["move"])[:, 0].astype(np.int64)
        stepped = move.copy()
        if "final_observation" in info:  # same-step auto-reset: the step's own obs is the terminal one
            for i in np.nonzero(info["_final_observation"])[0]:
                stepped[i] = int(np.asarray(info["final_observation"][i]["move"])[0])
        rows = np.ones(self.num_envs, dtype=bool) if rows is None else np.asarray(rows, dtype=bool)
        special = rows & (stepped != self._prev_move) & np.isin(stepped, SPECIALS)
        self._special += special
        self._special_neutral += special & ~np.isin(self._prev_move, NORMALS)
        self._prev_move[rows] = move[rows]  # after an auto-reset: the new episode's first move
        for i in np.nonzero(rows & (np.asarray(term) | np.asarray(trunc)))[0]:
            self._per_episode[i].append(int(self._special[i]))
            self._special[i] = 0

    def step(self, actions):
        res = self.env.step(actions)
        self._count(res[0], res[2], res[3], res[4])
        return res

    def step_masked(self, actions, active):
        res = self.env.step_masked(actions, active)
        self._count(res[0], res[2], res[3], res[4], rows=active)
        return res

    @property
    def metric_special_moves_per_episode(self):
        """Per arena, the special-move count of every finished episode."""
        return self._per_episode

    @property
    def metric_special_moves_from_neutral_per_episode(self):
        return self._neutral_per_episode

    def report(self):
        """Totals over all arenas (statistics.py:61-70), returned instead of printed."""
        eps = [c for arena in self._per_episode for c in arena]
        neutral = [c for arena in self._neutral_per_episode for c in arena]
        return {"episodes": len(eps), "special_moves_total": sum(eps),
                "special_moves_average": sum(eps) / len(eps) if eps else float("nan"),
                "special_moves_from_neutral_total": sum(neutral),
                "special_moves_from_neutral_average": sum(neutral) / len(eps) if eps else float("nan")}
