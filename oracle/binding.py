"""ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from footsies_gym_amd import _abi as abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


def build(force=False):
    if force or not os.path.exists(LIB_PATH) or any(
            os.path.getmtime(os.path.join(HERE, f)) > os.path.getmtime(LIB_PATH)
            for f in ("footsies_oracle.c", "or_tables.h")):
        subprocess.run(["make", "-C", HERE, "-B" if force else "liboracle.so"], check=True,
                       stdout=subprocess.DEVNULL)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.or_create.argtypes = [C.POINTER(abi.fs_config), C.POINTER(C.c_void_p)]
        L.or_reset.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.or_step.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_set_p2_mode.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.or_step_masked.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_step_n_hashed.argtypes = [C.c_void_p, C.c_int, C.c_uint64]
        L.or_outputs_get.argtypes = [C.c_void_p, C.POINTER(abi.fs_outputs)]
        L.or_get_env_state.argtypes = [C.c_void_p, C.POINTER(abi.fs_env_state)]
        L.or_get_state.argtypes = [C.c_void_p, C.POINTER(abi.fs_arena_state)]
        L.or_set_state.argtypes = [C.c_void_p, C.POINTER(abi.fs_arena_state)]
        L.or_destroy.argtypes = [C.c_void_p]
        L.or_hash_action.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_int]
        L.or_hash_action.restype = C.c_uint8
        L.or_set_threads.argtypes = [C.c_int]
        L.or_get_threads.restype = C.c_int
        _lib = L
    return _lib


def hash_actions(seed, n_envs, t, player):
    """Vectorised splitmix64 action stream, numpy-side."""
    M = np.uint64(0xFFFFFFFFFFFFFFFF)
    env = np.arange(n_envs, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = np.uint64(seed) ^ (env * np.uint64(0x9E3779B97F4A7C15)) ^ np.uint64((t << 1) | player)
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return (x & np.uint64(7)).astype(np.uint8)


class Oracle:
    """Host-side mirror of the fs_* API over the CPU oracle."""

    def __init__(self, num_envs, p2_mode=abi.FS_P2_EXTERNAL, dense_reward=True, float_mode=abi.FS_FLOAT_STRICT32,
                 autoreset_mode=abi.FS_AUTORESET_SAME_STEP, base_seed=0, frame_delay=0, p1_mode=abi.FS_P1_EXTERNAL,
                 arena_base=0):
        L = lib()
        cfg = abi.fs_config(num_envs=num_envs, device_id=-1, p2_mode=p2_mode, dense_reward=int(dense_reward),
                            frame_delay=frame_delay, float_mode=float_mode, autoreset_mode=autoreset_mode,
                            base_seed=base_seed, p1_mode=p1_mode, arena_base=arena_base)
        h = C.c_void_p()
        rc = L.or_create(C.byref(cfg), C.byref(h))
        if rc != 0:
            raise RuntimeError("or_create failed: %d" % rc)
        self.h = h
        self.n = num_envs
        self.cfg = cfg
        o = abi.fs_outputs()
        L.or_outputs_get(self.h, C.byref(o))
        self._out = {}
        for name, (dt, cols) in abi.OUTPUT_SPEC.items():
            ptr = getattr(o, name)
            nbytes = np.dtype(dt).itemsize * cols * num_envs
            buf = (C.c_uint8 * nbytes).from_address(ptr)
            a = np.frombuffer(buf, dtype=dt)
            self._out[name] = a.reshape(num_envs, cols) if cols > 1 else a

    def outputs(self, copy=True):
        return {k: (v.copy() if copy else v) for k, v in self._out.items()}

    def reset(self, seeds=None, mask=None, flags=abi.FS_RESET_IF_NEEDED):
        s = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint64)
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        rc = lib().or_reset(self.h, None if s is None else s.ctypes.data, None if m is None else m.ctypes.data,
                            flags)
        assert rc == 0, rc
        return self.outputs()

    def set_p2_mode(self, mode, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        return lib().or_set_p2_mode(self.h, mode, None if m is None else m.ctypes.data)

    def step(self, p1, p2=None, active=None):
        p1 = None if p1 is None else np.ascontiguousarray(p1, dtype=np.uint8)
        p2 = None if p2 is None else np.ascontiguousarray(p2, dtype=np.uint8)
        q1 = None if p1 is None else p1.ctypes.data
        q2 = None if p2 is None else p2.ctypes.data
        if active is None:
            rc = lib().or_step(self.h, q1, q2)
        else:
            m = np.ascontiguousarray(active, dtype=np.uint8)
            rc = lib().or_step_masked(self.h, q1, q2, m.ctypes.data)
        assert rc == 0, rc
        return self.outputs()

    def step_n_hashed(self, n, seed):
        rc = lib().or_step_n_hashed(self.h, n, seed)
        assert rc == 0, rc

    def env_state(self):
        arr = (abi.fs_env_state * self.n)()
        lib().or_get_env_state(self.h, arr)
        return np.ctypeslib.as_array(arr).copy()

    def state(self):
        arr = (abi.fs_arena_state * self.n)()
        lib().or_get_state(self.h, arr)
        return np.ctypeslib.as_array(arr).copy()

    def set_state(self, states):
        arr = (abi.fs_arena_state * self.n)()
        np.ctypeslib.as_array(arr)[:] = states
        return lib().or_set_state(self.h, arr)

    def close(self):
        if self.h:
            lib().or_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
