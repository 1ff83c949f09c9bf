"""FootsiesVectorEnv: the reference FootsiesEnv surface, vectorized over N arenas on one GPU.

Reference: footsies-gym/footsies_gym/envs/footsies.py (FE).  Per arena, the
observation, info, reward, termination and reset handshake are those of
``FootsiesEnv.reset`` / ``FootsiesEnv.step`` (FE:482-570); they are computed on
the GPU by libfootsies.so and only converted to the gymnasium dtypes here.

Differences from the reference, by design:
  * one object steps N arenas; actions are (N,3) booleans or (N,) ints 0..7;
  * no game process, sockets, fast-forward or sync modes -- the simulation is
    in-process and always "synced" (FE:44, 225-228);
  * auto-reset: ``autoreset_mode="same_step"`` follows gymnasium 0.29's
    SyncVectorEnv (returned obs is the new episode's first obs, the terminal one
    is in ``infos["final_observation"]``); ``"next_step"`` follows gymnasium 1.x.
"""
import ctypes as C

import numpy as np

from . import _abi, battle_state
from . import spaces as sp
from ._lib import FootsiesGameClosedError, check, lib
from .simulator import FootsiesSim, decode_actions, encode_actions

try:  # pragma: no cover - depends on the environment
    from gymnasium.vector import VectorEnv as _VectorEnvBase  # a gymnasium.vector.VectorEnv when importable
except Exception:  # gymnasium is not installed in this image
    _VectorEnvBase = object
try:
    from gymnasium import Env as _EnvBase  # FootsiesEnv is a gymnasium.Env when importable (FE:20)
except Exception:
    _EnvBase = object


_HEAP_RETAINED = False


def retain_host_heap():
    """Keep freed host memory in the process heap instead of returning it to the OS.

    A numpy step at 65 536 arenas allocates ~8 MB of fresh arrays (the int64 / float32 obs, the
    info copies FE:379 asks for, the action booleans).  glibc serves blocks that size by mmap and
    unmaps them on free, so every step re-faults every page of its arrays: measured in the build
    container, the host conversion of one step took 5.2 ms, 1.7 ms once glibc keeps blocks below
    256 MB on its heap (mallopt M_MMAP_THRESHOLD) and stops trimming the heap (M_TRIM_THRESHOLD).
    Process-wide and irreversible (freed memory up to 1 GB then stays resident in this process),
    so it is opt-in: call it, or create a numpy-output FootsiesVectorEnv with
    ``retain_host_heap=True``; FOOTSIES_NO_MALLOPT=1 refuses it.  Returns whether the settings
    were applied."""
    global _HEAP_RETAINED
    import os
    if _HEAP_RETAINED or os.environ.get("FOOTSIES_NO_MALLOPT") == "1":
        return _HEAP_RETAINED
    try:
        import ctypes
        libc = ctypes.CDLL("libc.so.6")
        M_TRIM_THRESHOLD, M_MMAP_THRESHOLD = -1, -3  # <malloc.h>
        _HEAP_RETAINED = bool(libc.mallopt(M_MMAP_THRESHOLD, 256 << 20)) and bool(libc.mallopt(M_TRIM_THRESHOLD,
                                                                                              1 << 30))
    except OSError:  # not glibc: nothing to tune
        _HEAP_RETAINED = False
    return _HEAP_RETAINED


_tune_heap = retain_host_heap  # (the constructor's flag of the same name shadows it there)

_SRC_DTYPES = {"guard": np.uint8, "move": np.uint8, "move_frame": np.float32, "position": np.float32,
               "reward": np.float64, "terminated": np.uint8, "truncated": np.uint8, "frame": np.int32,
               "action": np.uint8, "hitstun": np.uint8}
_HOST_THREADS = None


def host_threads():
    """Host threads fs_host_convert splits a step's conversion over: FOOTSIES_HOST_THREADS, else
    up to 8 of the process's CPUs."""
    global _HOST_THREADS
    if _HOST_THREADS is None:
        import os
        env = os.environ.get("FOOTSIES_HOST_THREADS")
        try:
            avail = len(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            avail = os.cpu_count() or 1
        _HOST_THREADS = max(1, int(env)) if env else max(1, min(8, avail))
    return _HOST_THREADS


# The destination arrays of one conversion, in the fs_host_arrays member order: (member, dtype,
# columns); all of them are views of one fresh block (one allocation and one pointer per call).
_DST = (("guard", np.int64, 2), ("move", np.int64, 2), ("move_frame", np.float32, 2), ("position", np.float32, 2),
        ("info_guard", np.int64, 2), ("info_move", np.int64, 2), ("info_move_frame", np.float32, 2),
        ("info_position", np.float32, 2), ("frame", np.int64, 0), ("p1_action", np.bool_, 3),
        ("p2_action", np.bool_, 3), ("p1_hitstun", np.int64, 0), ("p2_hitstun", np.int64, 0),
        ("reward", np.float64, 0), ("terminated", np.bool_, 0), ("truncated", np.bool_, 0))
_SRC_NAMES = ("guard", "move", "move_frame", "position", "frame", "action", "hitstun")
_STEP_NAMES = ("reward", "terminated", "truncated")
# (member, dtype, columns, bytes per row) of the destination members, in _DST order
_DST_ROWS = tuple((name, np.dtype(dt), c, np.dtype(dt).itemsize * max(c, 1)) for name, dt, c in _DST)
# (prefix, want_step) -> (weak references to the source arrays, their fs_outputs): the sim's pinned
# views are the same arrays every step, so their struct is built once
_SRC_STRUCTS = {}


def _src_struct(out, prefix, want_step):
    """fs_outputs over the source arrays of one conversion, and the converted copies it points into
    (to be kept alive over the call) when some source was not a C-contiguous array of its dtype."""
    import weakref
    arrs = [out[prefix + k] for k in _SRC_NAMES]
    if want_step:
        arrs += [out[k] for k in _STEP_NAMES]  # (step outputs carry no final_ variant)
    hit = _SRC_STRUCTS.get((prefix, want_step))
    if hit is not None and len(hit[0]) == len(arrs) and all(w() is a for w, a in zip(hit[0], arrs)):
        return hit[1], None
    keep, ptrs = [], {}
    for name, a in zip(_SRC_NAMES + (_STEP_NAMES if want_step else ()), arrs):
        if not (isinstance(a, np.ndarray) and a.dtype == _SRC_DTYPES[name] and a.flags.c_contiguous):
            a = np.ascontiguousarray(a, dtype=_SRC_DTYPES[name])
            keep.append(a)
        ptrs[name] = a.ctypes.data
    so = _abi.fs_outputs(**ptrs)
    if not keep:
        try:
            _SRC_STRUCTS[(prefix, want_step)] = (tuple(weakref.ref(a) for a in arrs), so)
        except TypeError:  # (an ndarray subclass without weak references: not cached)
            pass
    return so, keep


_DST_NO_COPIES = tuple(m for m in _DST_ROWS[:13] if not m[0].startswith("info_"))
# The destination members live in five blocks, one allocation each: the observation, the info,
# and the reward, terminated and truncated arrays on their own.  A caller that keeps one of a step's
# arrays (a rollout that appends `terminated`) holds only that array's block alive, not all ~9 MB of
# the step, whose blocks the next step then reuses.
_BLOCK_OF = {"guard": 0, "move": 0, "move_frame": 0, "position": 0, "reward": 2, "terminated": 3, "truncated": 4}


def _host_convert(out, prefix, rows, n, want_step, info_copies=True):
    """(obs, info[, (reward, terminated, truncated)]) of n rows of host outputs through
    fs_host_convert (one pass over the rows on the library's host threads).  info_copies=False:
    the info gets no observation entries (the caller shares the obs rows, see
    step_result_from_outputs)."""
    obs, info, extra, _ = _host_convert_on(out, prefix, rows, n, want_step, info_copies, start=False)
    return obs, info, extra


def _host_convert_on(out, prefix, rows, n, want_step, info_copies=True, start=False):
    """_host_convert; start=True returns as soon as the conversion runs on the library's threads
    (fs_host_convert_start), with a fourth result to keep alive until fs_host_convert_wait."""
    so, keep = _src_struct(out, prefix, want_step)
    members = _DST_ROWS if want_step else (_DST_ROWS[:13] if info_copies else _DST_NO_COPIES)
    offs, totals = [], [0, 0, 0, 0, 0]
    for m in members:  # 64-B aligned members of their block
        b = _BLOCK_OF.get(m[0], 1)
        offs.append((b, totals[b]))
        totals[b] += (n * m[3] + 63) & ~63
    blocks = [np.empty(t or 1, np.uint8) for t in (totals if want_step else totals[:2])]
    bases = [blk.ctypes.data for blk in blocks]
    if info_copies:
        dst = _abi.fs_host_arrays(*[bases[b] + off for b, off in offs])
    else:  # (the info_ members stay null: fs_host_convert skips them)
        dst = _abi.fs_host_arrays(**{m[0]: bases[b] + off for m, (b, off) in zip(members, offs)})
    views = {name: np.ndarray((n, c) if c else (n,), dt, blocks[b], off)
             for (name, dt, c, _), (b, off) in zip(members, offs)}
    r = None if rows is None else np.ascontiguousarray(rows, dtype=np.int64)
    n_src = len(out[prefix + "frame"])
    convert = lib().fs_host_convert_start if start else lib().fs_host_convert
    check(convert(C.byref(so), n_src, None if r is None else r.ctypes.data, n, C.byref(dst), host_threads()))
    hold = (keep, r) if start else None  # (the converted sources and rows live until the wait)
    obs = {k: views[k] for k in ("guard", "move", "move_frame", "position")}
    info = {k: views[k] for k in ("frame", "p1_action", "p2_action", "p1_hitstun", "p2_hitstun")}
    if info_copies:
        info.update({k: views["info_" + k] for k in ("guard", "move", "move_frame", "position")})  # FE:379's copies
    extra = (views["reward"], views["terminated"], views["truncated"]) if want_step else None
    return obs, info, extra, hold


def obs_info_from_outputs(out, prefix=""):
    """Host-side view of one set of kernel outputs -> (obs, info) batches with the
    reference dtypes: MultiDiscrete -> int64, Box -> float32 (FE:157-168, 336-380); converted
    by fs_host_convert (obs_info_from_outputs_numpy is the same in numpy)."""
    n = len(out[prefix + "frame"])
    obs, info, _ = _host_convert(out, prefix, None, n, False)
    return obs, info


def obs_info_from_outputs_numpy(out, prefix=""):
    """obs_info_from_outputs written with numpy ops (the reference the native conversion is
    tested against)."""
    obs = {  # (always new arrays: ``out`` may be views of a reused host buffer)
        "guard": np.array(out[prefix + "guard"], dtype=np.int64),
        "move": np.array(out[prefix + "move"], dtype=np.int64),
        "move_frame": np.array(out[prefix + "move_frame"], dtype=np.float32),
        "position": np.array(out[prefix + "position"], dtype=np.float32),
    }
    act = decode_actions(out[prefix + "action"])  # (N, 2, 3): both players in one pass
    hs = np.asarray(out[prefix + "hitstun"], dtype=np.int64)
    info = {
        "frame": np.asarray(out[prefix + "frame"], dtype=np.int64),
        "p1_action": act[:, 0],
        "p2_action": act[:, 1],
        "p1_hitstun": hs[:, 0],
        "p2_hitstun": hs[:, 1],
    }
    info.update({k: v.copy() for k, v in obs.items()})  # FE:379 puts a copy of the obs in the info
    return obs, info


def step_result_from_outputs(out, autoreset_mode="same_step"):
    """(obs, rewards, terminations, truncations, infos) from host copies of the outputs: one
    fs_host_convert pass over all rows -- running on the library's threads while this thread
    builds the terminated arenas' final-observation dicts (fs_host_convert_start / _wait) -- and one
    over the terminated arenas' final records."""
    n = len(out["frame"])
    if n < _ASYNC_MIN_ROWS:  # (fs_host_convert runs these on the calling thread anyway)
        obs, info, (rewards, term, trunc) = _host_convert(out, "", None, n, True)
        _final_entries(out, info, autoreset_mode)
        return obs, rewards, term, trunc, info
    obs, info, (rewards, term, trunc), hold = _host_convert_on(out, "", None, n, True, start=True)
    try:
        _final_entries(out, info, autoreset_mode)
    finally:
        check(lib().fs_host_convert_wait())
        del hold
    return obs, rewards, term, trunc, info


# below this many rows fs_host_convert converts on the calling thread (fs_api.cpp host_convert_run),
# and handing the conversion to the library's runner thread would only add its wake-up
_ASYNC_MIN_ROWS = 8192


def _final_entries(out, info, autoreset_mode):
    """info's final_observation / final_info entries (gymnasium 0.29) of the arenas the step ended,
    from the source outputs (the step's converted arrays may still be in conversion)."""
    if autoreset_mode != "same_step":
        return
    term = np.asarray(out["terminated"]) != 0
    if term.any():
        idx = np.nonzero(term)[0]
        # only the terminated arenas' final outputs are converted
        fobs, finfo, _ = _host_convert(out, "final_", idx, len(idx), False, info_copies=False)
        for a in fobs.values():  # shared by final_observation and final_info below: read-only rows
            a.setflags(write=False)
        final_obs = np.empty(len(term), dtype=object)
        final_info = np.empty(len(term), dtype=object)
        # Per-arena dicts (gymnasium 0.29's contract: one dict per terminated env, None elsewhere),
        # their values the rows of the batched final arrays: list(a) makes every row view in one C
        # loop, and literal dicts are built without a zip per entry.  An arena's final info holds
        # the same observation rows as its final observation, as FE:379's `**obs` puts the obs
        # dict's own values (tuples) into the reference's info.
        g, m, mf, pos = (list(fobs[k]) for k in ("guard", "move", "move_frame", "position"))
        final_obs[idx] = [{"guard": a, "move": b, "move_frame": c, "position": d} for a, b, c, d in zip(g, m, mf, pos)]
        fr, a1, a2, h1, h2 = (list(finfo[k]) for k in ("frame", "p1_action", "p2_action", "p1_hitstun", "p2_hitstun"))
        final_info[idx] = [{"frame": v0, "p1_action": v1, "p2_action": v2, "p1_hitstun": v3, "p2_hitstun": v4,
                            "guard": v5, "move": v6, "move_frame": v7, "position": v8}
                           for v0, v1, v2, v3, v4, v5, v6, v7, v8 in zip(fr, a1, a2, h1, h2, g, m, mf, pos)]
        info["final_observation"] = final_obs
        info["_final_observation"] = term.copy()
        info["final_info"] = final_info
        info["_final_info"] = term.copy()


class FootsiesVectorEnv(_VectorEnvBase):
    """N FOOTSIES arenas as one vector environment (a ``gymnasium.vector.VectorEnv`` subclass
    whenever gymnasium is importable; its reset / step / close are overridden here, so neither
    0.29's async hooks nor 1.x's base methods are used).

    Parameters follow FootsiesEnv.__init__ (FE:34-53) where they still have a
    meaning: ``frame_delay`` (observations and info ``frame_delay`` steps old, FE:126-131,
    532-535; reward and termination current), ``dense_reward``, ``opponent``:
      * ``None`` -> the in-game scripted bot as P2 (FE:236-237, ``--p2-bot``);
      * a callable ``opponent(obs, info) -> actions`` -> P2 driven by that policy,
        called every step with the most recent batched obs/info (FE:525-527);
        ``set_opponent`` can then switch arenas between it and the bot (FE:458-480);
      * ``"noop"`` -> P2 never presses anything;
    ``by_example`` (FE:83-84, 118, 230-232): the in-game bot plays P1 as well and the agent only
    observes -- ``step`` ignores its actions (FE:522-523).
    ``output="torch"`` returns device tensors (zero-copy) instead of numpy.
    ``retain_host_heap=True`` (numpy output, opt-in): tune glibc for the step's large fresh arrays
    (``retain_host_heap()``: mallopt M_MMAP_THRESHOLD 256 MB, M_TRIM_THRESHOLD 1 GB) -- process-wide,
    so off by default; at 65 536 arenas it saves the re-faulting of ~9 MB of pages per step.
    (``_host_outputs``, internal, numpy output only: the kernels write the outputs into pinned host
    memory -- FootsiesSim ``host_outputs`` -- instead of HBM, so a step needs no device-to-host copy
    of its own.  The default for numpy output: at 65 536 arenas a step took 0.45-0.46 ms so, against
    0.50-0.51 ms with the outputs in HBM and one copy a step (profiles/r04p_venv_pieces.txt).)
    """

    metadata = {"render_modes": [], "render_fps": 60}
    render_mode = None
    spec = None
    is_vector_env = True

    def __init__(self, num_envs, device=0, opponent=None, dense_reward=True, frame_delay=0,
                 autoreset_mode="same_step", float_mode="strict", seed=0, vs_player=False, by_example=False,
                 output="numpy", retain_host_heap=False, _host_outputs=None):
        if vs_player:
            raise ValueError("vs_player needs a human at the game window; not available in the simulator")
        if not 0 <= int(frame_delay) <= _abi.FS_MAX_FRAME_DELAY:
            raise ValueError("frame_delay must be in [0, %d]" % _abi.FS_MAX_FRAME_DELAY)
        if output not in ("numpy", "torch"):
            raise ValueError("output must be 'numpy' or 'torch'")
        if _host_outputs is None:
            _host_outputs = output == "numpy"
        if _host_outputs and output != "numpy":
            raise ValueError("host-memory outputs serve the numpy output only")
        self.num_envs = int(num_envs)
        self.output = output
        if output == "numpy" and retain_host_heap:
            _tune_heap()
        self.autoreset_mode = autoreset_mode
        self.dense_reward = dense_reward
        self._opponent = opponent
        p2 = "bot" if opponent is None else ("noop" if isinstance(opponent, str) and opponent == "noop" else "external")
        if p2 == "external" and not callable(opponent):
            raise ValueError("opponent must be None, 'noop' or a callable(obs, info) -> actions")
        self.by_example = bool(by_example)
        self.sim = FootsiesSim(self.num_envs, device=device, p2_mode=p2, dense_reward=dense_reward,
                               float_mode=float_mode, autoreset_mode=autoreset_mode, seed=seed,
                               frame_delay=frame_delay, p1_mode="bot" if by_example else "external",
                               host_outputs=_host_outputs)
        self._p2_bot = np.zeros(self.num_envs, dtype=bool)  # arenas switched to the bot (set_opponent)
        self._all_bot = False  # == self._p2_bot.all(), kept beside it (step reads it every call)
        self.single_observation_space = sp.single_observation_space()
        self.single_action_space = sp.single_action_space()
        self.observation_space = sp.batch_observation_space(self.num_envs)
        self.action_space = sp.batch_action_space(self.num_envs)
        self.reward_range = (-1, 1)
        self.closed = False
        self._last = None  # most recent (obs, info) for the opponent callable

    # -- gymnasium.vector.VectorEnv API ---------------------------------------------------
    def reset(self, *, seed=None, options=None):
        """FootsiesEnv.reset on every arena (or ``options["mask"]``).  ``seed``: int (arena i
        gets seed + i) or a sequence of N seeds -> Random.InitState of each arena's bot.
        ``options["hard"]=True`` forces the RESET command even after a terminated step."""
        self._check_open()
        options = options or {}
        seeds = None
        if seed is not None:
            seeds = (np.asarray(seed, dtype=np.uint64) if np.ndim(seed) else
                     np.uint64(seed) + np.arange(self.num_envs, dtype=np.uint64))
        out = self.sim.reset(seeds=seeds, mask=options.get("mask"), hard=bool(options.get("hard", False)))
        if self.output == "torch":
            self._last = (out, None)
            return {k: out[k] for k in ("guard", "move", "move_frame", "position")}, out
        obs, info = obs_info_from_outputs(self.sim.outputs_numpy(copy=False, _synced=True))  # (reset waited)
        self._last = (obs, info)
        return obs, info

    def set_opponent(self, opponent, mask=None):
        """FootsiesEnv.set_opponent (FE:458-480): P2 of every arena (or of ``mask``) becomes the
        callable ``opponent(obs, info) -> actions``, or the in-game bot for ``None`` -- the P2_BOT
        command, sent only when the arena's P2 changes between the two kinds.  Like the reference,
        it needs an environment created with a custom opponent (else RuntimeError) and returns
        None.  A bot keeps its queues, FightState and last answer while a callable plays, and is
        never Reset after being switched in (see fs_set_p2_mode)."""
        if self.sim.p2_mode != "external":
            raise RuntimeError("the environment needs to be created with a custom opponent before calling this method")
        if opponent is not None and not callable(opponent):
            raise ValueError("opponent must be None or a callable(obs, info) -> actions")
        sel = np.ones(self.num_envs, dtype=bool) if mask is None else np.asarray(mask, dtype=bool).reshape(-1)
        if opponent is None:
            change = sel & ~self._p2_bot
            if change.any():
                self.sim.set_p2_mode("bot", change)
            self._p2_bot |= sel
            self._all_bot = bool(self._p2_bot.all())
        else:
            change = sel & self._p2_bot
            if change.any():
                self.sim.set_p2_mode("external", change)
            self._p2_bot &= ~sel
            self._all_bot = bool(self._p2_bot.all())
            self._opponent = opponent

    def _p2_actions(self):
        """P2's actions for a remote P2 (FE:525-527); arenas whose P2 is the bot ignore theirs."""
        if self.sim.p2_mode != "external":
            return None
        if self._all_bot or self._opponent is None or self._last is None:
            return np.zeros(self.num_envs, np.uint8)
        return self._opponent(*self._last)

    def _check_open(self):
        if self.closed:
            raise FootsiesGameClosedError("the environment was closed")

    def step(self, actions):
        self._check_open()
        p2 = self._p2_actions()
        if self.by_example:
            actions = None  # FE:522-523: the bot plays P1, the agent's action is not sent
        out = self.sim.step(actions, p2)
        if self.output == "torch":
            obs = {k: out[k] for k in ("guard", "move", "move_frame", "position")}
            self._last = (obs, out)
            return obs, out["reward"], out["terminated"], out["truncated"], out
        obs, rew, term, trunc, info = step_result_from_outputs(self.sim.outputs_numpy(copy=False, _synced=True),
                                                               self.autoreset_mode)  # (step waited)
        self._last = (obs, info)
        return obs, rew, term, trunc, info

    def step_masked(self, actions, active):
        """Step only the arenas where ``active`` is true (fs_step_masked), as separate
        FootsiesEnv instances that are stepped at different times.  The returned batch
        holds, for inactive arenas, their previous observation with reward 0 and not
        terminated (numpy output)."""
        self._check_open()
        p2 = self._p2_actions()
        if self.by_example:
            actions = None
        out = self.sim.step(actions, p2, active=active)
        if self.output == "torch":
            obs = {k: out[k] for k in ("guard", "move", "move_frame", "position")}
            self._last = (obs, out)
            return obs, out["reward"], out["terminated"], out["truncated"], out
        host = self.sim.outputs_numpy()
        idle = ~np.asarray(active, dtype=bool).reshape(self.num_envs)
        host["reward"][idle] = 0.0
        host["terminated"][idle] = 0
        host["truncated"][idle] = 0
        obs, rew, term, trunc, info = step_result_from_outputs(host, self.autoreset_mode)
        self._last = (obs, info)
        return obs, rew, term, trunc, info

    def close(self, **kwargs):
        sim = getattr(self, "sim", None)  # (also from a base-class __del__ after a failed __init__)
        if sim is not None and not getattr(self, "closed", False):
            sim.close()
        self.closed = True

    # -- FootsiesEnv extras (FE:432-480) ------------------------------------------------
    def save_battle_state(self):
        """STATE_SAVE (BC:148-151): canonical per-arena state, see fs_arena_state."""
        return self.sim.get_state()

    def load_battle_state(self, state):
        """STATE_LOAD (BC:153-156) of canonical states (which carry each arena's P2 actor)."""
        self.sim.set_state(state)
        if self.sim.p2_mode == "external":
            self._p2_bot = np.asarray(state["p2_bot"], dtype=bool).copy()
            self._all_bot = bool(self._p2_bot.all())

    def save_battle_state_json(self, arena=0):
        """STATE_SAVE of one arena in the reference's BattleState JSON (battle_state.py)."""
        return battle_state.dumps(battle_state.battle_state(self.sim.get_state(), arena))

    def load_battle_state_json(self, state, arena=0):
        """STATE_LOAD of one arena from BattleState JSON text, a dict or a FootsiesBattleState;
        the arena keeps what BattleState does not carry (bot RNG, recording, reward sum)."""
        if isinstance(state, battle_state.FootsiesBattleState):
            state = state.to_dict()
        states = self.sim.get_state()
        self.sim.set_state(battle_state.load_into(states, arena, state))

    @property
    def most_recent_observation(self):
        return None if self._last is None else self._last[0]

    @property
    def most_recent_info(self):
        return None if self._last is None else self._last[1]

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class FootsiesEnv(_EnvBase):
    """Single-environment adapter with the reference FootsiesEnv API (FE:20-578) over
    one arena: tuples of Python ints/floats in, reference-shaped dicts out.  A
    ``gymnasium.Env`` subclass whenever gymnasium is importable (its reset / step / close are
    overridden here)."""

    metadata = {"render_modes": "human", "render_fps": 60}
    render_mode = None  # rendering is the Unity window's (out of scope)
    spec = None

    VALID_SYNC_MODES = frozenset({"async", "synced_non_blocking", "synced_blocking"})

    def __init__(self, frame_delay=0, render_mode=None, game_path="./Build/FOOTSIES", game_address="localhost",
                 game_port=11000, skip_instancing=False, fast_forward=True, fast_forward_speed=6.0,
                 sync_mode="synced_non_blocking", remote_control_port=11002, by_example=False, opponent=None,
                 opponent_port=11001, vs_player=False, dense_reward=True, log_file=None, log_file_overwrite=False,
                 device=0, seed=0):
        """The reference's constructor (FE:34-53), in its order, plus ``device`` / ``seed``.  The
        arguments that configure the game process and its sockets (game_path .. remote_control_port,
        opponent_port, log_file*) are validated and recorded as FE does, and have no effect: the
        game is the in-process simulator, always stepped in lockstep with the agent."""
        # FE:100-108, same checks in the same order and the same exceptions
        if sync_mode not in self.VALID_SYNC_MODES:
            raise ValueError("sync mode '%s' is invalid, must be one of %s" % (sync_mode, set(self.VALID_SYNC_MODES)))
        if opponent is not None and vs_player:
            raise ValueError("custom opponent and human opponent can't be specified together")
        if vs_player:  # a human P2 needs the game window (out of scope)
            raise ValueError("vs_player=True needs a human at the game window; the simulator has no human P2")
        self.game_path, self.game_address, self.game_port = game_path, game_address, game_port
        self.skip_instancing, self.fast_forward, self.fast_forward_speed = skip_instancing, fast_forward, fast_forward_speed
        self.sync_mode, self.remote_control_port, self.opponent_port = sync_mode, remote_control_port, opponent_port
        self.by_example, self.vs_player, self.dense_reward = by_example, vs_player, dense_reward
        self.log_file, self.log_file_overwrite = log_file, log_file_overwrite
        # FE:133-134; "human" rendering is the Unity window's: accepted and recorded, nothing is drawn
        assert render_mode is None or render_mode in self.metadata["render_modes"]
        self.render_mode = render_mode
        self._opp = opponent
        # next_step auto-reset keeps FE's handshake: a terminal step() returns the terminal
        # obs and the agent's reset() then finds the game already at state(-1) (no RESET)
        # (one arena: the kernels write its outputs straight into pinned host memory, FootsiesSim
        # host_outputs, so a step costs one launch and one stream synchronize, no copies)
        self.venv = FootsiesVectorEnv(1, device=device, opponent=self._wrap(opponent), dense_reward=dense_reward,
                                      frame_delay=frame_delay, seed=seed, autoreset_mode="next_step",
                                      by_example=by_example, _host_outputs=True)
        self.observation_space = self.venv.single_observation_space
        self.action_space = self.venv.single_action_space
        self.reward_range = (-1, 1)
        self._most_recent_observation = None
        self._most_recent_info = None

    @staticmethod
    def _py(obs, info):
        def pos(x):  # EnvironmentState floats travel as shortest round-trip JSON text (FE:319)
            return float(str(np.float32(x)))
        o = {"guard": tuple(int(v) for v in obs["guard"][0]), "move": tuple(int(v) for v in obs["move"][0]),
             "move_frame": tuple(int(v) for v in obs["move_frame"][0]),
             "position": tuple(pos(v) for v in obs["position"][0])}
        i = {"frame": int(info["frame"][0]), "p1_action": tuple(bool(v) for v in info["p1_action"][0]),
             "p2_action": tuple(bool(v) for v in info["p2_action"][0]), "p1_hitstun": int(info["p1_hitstun"][0]),
             "p2_hitstun": int(info["p2_hitstun"][0]), **o}
        return o, i

    def _wrap(self, opponent):
        """A reference opponent (obs, info) -> (left, right, attack) over the single-arena dicts
        (FE:525-527: it sees the agent's most recent observation and info)."""
        if opponent is None:
            return None
        return lambda obs, info: np.array([encode_actions([opponent(self._most_recent_observation,
                                                                    self._most_recent_info)])[0]], np.uint8)

    def set_opponent(self, opponent):
        """FE:458-480: switch P2 between the custom opponent and the in-game bot (None).  Needs an
        environment created with a custom opponent (RuntimeError otherwise); returns None."""
        self.venv.set_opponent(self._wrap(opponent))
        self._opp = opponent

    def reset(self, *, seed=None, options=None):
        obs, info = self.venv.reset(seed=seed, options=options)
        o, i = self._py(obs, info)
        self._most_recent_observation, self._most_recent_info = dict(o), dict(i)
        return o, i

    @staticmethod
    def _py_host(h):
        """_py of the one arena straight from the host copy of the outputs (the values that
        step_result_from_outputs + _py produce, without the batch arrays in between)."""
        def pos(x):
            return float(str(np.float32(x)))
        g, m, mf, p = h["guard"][0].tolist(), h["move"][0].tolist(), h["move_frame"][0].tolist(), h["position"][0].tolist()
        a1, a2 = h["action"][0].tolist()
        hs = h["hitstun"][0].tolist()
        o = {"guard": (g[0], g[1]), "move": (m[0], m[1]), "move_frame": (int(mf[0]), int(mf[1])),
             "position": (pos(p[0]), pos(p[1]))}
        i = {"frame": int(h["frame"][0]), "p1_action": (a1 & 1 != 0, a1 & 2 != 0, a1 & 4 != 0),
             "p2_action": (a2 & 1 != 0, a2 & 2 != 0, a2 & 4 != 0), "p1_hitstun": hs[0], "p2_hitstun": hs[1], **o}
        return o, i

    def step(self, action):
        # the one-arena path of FootsiesVectorEnv.step (next-step auto-reset: no final_* outputs),
        # converted from the host buffer directly (tests/test_gpu_api.py holds it to the batch path)
        v = self.venv
        v._check_open()
        p2 = v._p2_actions()
        v.sim.step(None if v.by_example else np.asarray([action]).reshape(1, 3), p2)
        h = v.sim.outputs_numpy(copy=False, _synced=True)  # (step waited for the host outputs)
        o, i = self._py_host(h)
        v._last = (o, i)  # (the wrapped opponent reads this env's most recent dicts, not these)
        self._most_recent_observation, self._most_recent_info = dict(o), dict(i)
        return o, float(h["reward"][0]), bool(h["terminated"][0]), False, i

    def close(self):
        self.venv.close()

    def save_battle_state(self):
        """FE:466-471: the game's BattleState (STATE_SAVE)."""
        return battle_state.FootsiesBattleState.from_json(self.venv.save_battle_state_json(0))

    def load_battle_state(self, state):
        """FE:473-478: STATE_LOAD of a FootsiesBattleState."""
        self.venv.load_battle_state_json(state, 0)

    @property
    def most_recent_observation(self):
        return self._most_recent_observation

    @staticmethod
    def find_ports(start, step=1, stop=None):
        """FE:590-614: three TCP ports not in use (game, opponent, remote control), scanning from
        `start` by `step` (up to `stop`).  This environment opens no sockets; the ports matter to
        scripts that start several reference-style instances, or the wire server (server.py)."""
        import itertools
        import psutil
        used = {c.laddr.port for c in psutil.net_connections(kind="tcp4") if c.laddr}
        candidates = itertools.count(start, step) if stop is None else range(start, stop, step)
        free = list(itertools.islice((q for q in candidates if q not in used), 3))
        if len(free) < 3:
            raise RuntimeError("could not find 3 free ports for a new FOOTSIES instance (starting at %d with steps "
                               "of %d until %s)" % (start, step, stop))
        return {"game_port": free[0], "opponent_port": free[1], "remote_control_port": free[2]}

    @property
    def most_recent_info(self):
        return self._most_recent_info
