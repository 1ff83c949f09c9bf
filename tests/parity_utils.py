"""Helpers shared by the parity tests: bitwise comparison of output/state arrays."""
import numpy as np

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
