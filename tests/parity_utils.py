"""Helpers shared by the parity tests: bitwise comparison of output/state arrays."""
import numpy as np

from footsies_gym_amd import _abi

OBS_KEYS = ("guard", "move", "move_frame", "position", "reward", "terminated", "truncated", "frame", "action",
            "hitstun")
FINAL_KEYS = ("final_guard", "final_move", "final_move_frame", "final_position", "final_frame", "final_action",
              "final_hitstun")


def bits(a):
    a = np.ascontiguousarray(a)
    if a.dtype.kind == "f":
        return a.view({4: np.uint32, 8: np.uint64}[a.dtype.itemsize])
    return a


def assert_same(name, expected, got, step=None, extra=""):
    e, g = bits(np.asarray(expected)), bits(np.asarray(got))
    if e.shape != g.shape or not np.array_equal(e, g):
        bad = np.argwhere(e != g) if e.shape == g.shape else None
        where = "" if bad is None or len(bad) == 0 else " first mismatch at %s: expected %r got %r" % (
            tuple(bad[0]), np.asarray(expected)[tuple(bad[0])], np.asarray(got)[tuple(bad[0])])
        raise AssertionError("%s differs%s%s %s" % (name, "" if step is None else " at step %d" % step, where, extra))


def compare_outputs(expected, got, step=None, same_step=True):
    for k in OBS_KEYS:
        assert_same(k, expected[k], got[k], step)
    if same_step:
        term = np.asarray(expected["terminated"]).astype(bool)
        for k in FINAL_KEYS:
            assert_same(k, np.asarray(expected[k])[term], np.asarray(got[k])[term], step)


def compare_states(expected, got, step=None):
    """Field-by-field comparison of fs_arena_state structured arrays."""
    for name in expected.dtype.names:
        if name.startswith("pad"):
            continue
        if name == "f":
            for fname in expected["f"].dtype.names:
                if fname.startswith("pad"):
                    continue
                assert_same("f." + fname, expected["f"][fname], got["f"][fname], step)
        else:
            assert_same(name, expected[name], got[name], step)


ACTION_FRAMES = {0: 24, 1: 24, 2: 24, 10: 16, 11: 22, 100: 22, 105: 21, 110: 44, 115: 55, 200: 17, 301: 23,
                 305: 15, 306: 15, 310: 36, 350: 1, 500: 500, 510: 33}  # frameCount per actionID (data/f00.json)
LOOPING = {0, 1, 2, 350, 510}
MOVE_PLAN_LEN, ATTACK_PLAN_LEN = [30, 90, 56, 70, 33, 60, 63], [30, 19, 23, 61, 121]


def random_bot_fields(n, rng, prefix=""):
    """Arbitrary queues mid-plan and FightState of one BattleAI (canonical fs_arena_state fields)."""
    ids = np.array(sorted(ACTION_FRAMES), dtype=np.int32)
    mp = rng.integers(-1, 7, n)
    ap = rng.integers(-1, 5, n)
    return {prefix + "move_plan": mp, prefix + "attack_plan": ap,
            prefix + "move_index": np.where(mp < 0, 0, (rng.random(n) * np.take(MOVE_PLAN_LEN, np.maximum(mp, 0))).astype(int)),
            prefix + "attack_index": np.where(ap < 0, 0, (rng.random(n) * np.take(ATTACK_PLAN_LEN,
                                                                                   np.maximum(ap, 0))).astype(int)),
            prefix + "prev_distance": rng.uniform(0.0, 9.0, n).astype(np.float32),
            prefix + "prev_opponent_action": rng.choice(ids, n)}


def random_states(n, rng, p2="external", p2_bot_frac=0.0, geom_frac=0.0):
    """Arbitrary loadable arena states (fs_arena_state), not only ones reachable from a reset:
    any action at any frame up to its frameCount, buffered / reserved actions, hitstun, latches,
    hasWon, saturated recordings, random histories and bot queues -- the paths a played match
    reaches rarely (the hasWon request, reserve / buffer takes, DEAD past frame 63).  The actors
    fit the handle's P2 mode: a bot-created P2 is the bot and ready; with a remote P2 a fraction
    `p2_bot_frac` of the arenas has the bot switched in (bot_ready random: a never-Reset bot).
    `geom_frac` of the fighters are loaded off the ground (position.y in +-1.5, some exact box
    edges) and, independently, with a flipped facing (the general-geometry tick)."""
    st = np.zeros(n, dtype=np.ctypeslib.as_array((_abi.fs_arena_state * 1)()).dtype)
    ids = np.array(sorted(ACTION_FRAMES), dtype=np.int32)
    for k in range(2):
        f = st["f"][:, k]
        f["position_x"] = rng.uniform(-4.5, 4.5, n).astype(np.float32)
        f["action_id"] = rng.choice(ids, n)
        top = np.array([ACTION_FRAMES[a] - (1 if a in LOOPING else 0) for a in f["action_id"]])
        f["action_frame"] = (rng.random(n) * (top + 1)).astype(np.int32)
        f["hit_count"] = rng.integers(0, 3, n)
        f["hitstun"] = np.where(rng.random(n) < 0.5, 0, rng.integers(0, 31, n))
        f["vital"] = (rng.random(n) < 0.95).astype(np.int32)
        f["guard"] = rng.integers(0, 4, n)
        f["buffer_action_id"] = np.where(rng.random(n) < 0.6, -1, rng.choice(ids, n))
        f["reserve_action_id"] = np.where(rng.random(n) < 0.7, -1, rng.choice(ids, n))
        f["input_dir_history"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        f["attack_hold"] = rng.integers(0, 64, n)
        f["is_input_backward"] = rng.integers(0, 2, n)
        f["is_reserve_proximity_guard"] = rng.integers(0, 2, n)
        f["has_won"] = (rng.random(n) < 0.1).astype(np.uint8)
        if geom_frac:
            y = rng.choice(np.array([0.25, -0.25, 0.5, 1.0, -1.2, 0.1], np.float32), n)
            y = np.where(rng.random(n) < 0.5, y, rng.uniform(-1.5, 1.5, n).astype(np.float32))
            f["position_y"] = np.where(rng.random(n) < geom_frac, y, np.float32(0.0)).astype(np.float32)
            f["facing_flipped"] = (rng.random(n) < geom_frac).astype(np.uint8)
    st["frame_count"] = rng.integers(0, 5000, n)
    st["recording_count"] = np.where(rng.random(n) < 0.2, 18000, rng.integers(0, 18000, n))
    st["recording_last"] = rng.integers(0, 8, (n, 2))
    st["actor_input"] = rng.integers(0, 8, (n, 2))
    st["cumulative_reward"] = rng.integers(-3, 4, n) * 0.3
    st["rng"] = rng.integers(1, 2**32, (n, 4), dtype=np.uint64).astype(np.uint32)
    for k, v in {**random_bot_fields(n, rng), **random_bot_fields(n, rng, "p1_")}.items():
        st[k] = v
    st["bot_ready"] = rng.integers(0, 2, (n, 2))
    st["bot_input"] = rng.integers(0, 8, (n, 2))
    if p2 == "bot":
        st["p2_bot"] = 1
        st["bot_ready"][:, 1] = 1
    elif p2 == "external":
        st["p2_bot"] = (rng.random(n) < p2_bot_frac).astype(np.uint8)
    # a bot that is not ready has no FightState: canonical zeros (STAND)
    for k, pre in ((0, "p1_"), (1, "")):
        idle = st["bot_ready"][:, k] == 0
        st[pre + "prev_distance"][idle] = 0.0
        st[pre + "prev_opponent_action"][idle] = 0
    return st


def fused_kernel(name, n_envs, same_step=True, mi355x_simds=1024):
    """The name fs_step_kernel gives a two-lane fused row launch (`name`, e.g. "fsk::k_step_n<0, 0>")
    over n_envs arenas: the request-prefetch kernel (`..._pf`) at one wave per SIMD or less with
    same-step auto-reset (fs_kernels.hip request_prefetch; FOOTSIES_PREFETCH=0 / 1 forces it)."""
    import os
    forced = os.environ.get("FOOTSIES_PREFETCH", "")
    on = forced == "1" or (forced != "0" and (2 * n_envs + 63) // 64 <= mi355x_simds)
    if not same_step or "<" not in name or ", 3>" in name:  # (next-step auto-reset, per-arena actors: never)
        return name
    return name.replace("<", "_pf<", 1) if on else name
