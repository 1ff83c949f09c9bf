"""FootsiesSim: a thin, zero-copy handle over libfootsies.so for N arenas on one GPU.

PyTorch is used only as device-memory and stream plumbing: the output buffers are
torch tensors bound into the library (``fs_bind_outputs``) and the library runs
on torch's current stream (``fs_set_stream``), so device-side actions produced
by a policy and the observations consumed by it need no extra synchronisation.

Without torch (``backend="native"``, the default when torch is not installed) a handle with
``host_outputs`` still works: its outputs live in pinned host memory the library allocates
(``fs_host_alloc``), actions come from host arrays, and the library issues on its own stream --
what the numpy ``FootsiesVectorEnv`` / ``FootsiesEnv`` need, so a reference user with only numpy
(and gymnasium) can step the simulator.  The device-tensor APIs (step_n, trajectories, torch
outputs) need torch.
"""
import ctypes as C

import numpy as np

from . import _abi
from ._lib import check, lib

P2_MODES = {"external": _abi.FS_P2_EXTERNAL, "bot": _abi.FS_P2_BOT, "noop": _abi.FS_P2_NOOP}
P1_MODES = {"external": _abi.FS_P1_EXTERNAL, "bot": _abi.FS_P1_BOT}
FLOAT_MODES = {"strict": _abi.FS_FLOAT_STRICT32, "double": _abi.FS_FLOAT_DOUBLE}
AUTORESET_MODES = {"same_step": _abi.FS_AUTORESET_SAME_STEP, "next_step": _abi.FS_AUTORESET_NEXT_STEP}

_TORCH_DTYPES = {"u1": "uint8", "f4": "float32", "f8": "float64", "i4": "int32"}


def _torch():
    import torch
    return torch


def _torch_or_none():
    try:
        import torch
    except ImportError:
        return None
    return torch


def encode_actions(actions):
    """(N,3) booleans (left, right, attack) or (N,) ints 0..7 -> uint8 3-bit inputs.

    Mirrors TrainingRemoteActor.RequestTrainingInput (TrainingRemoteActor.cs:112-116):
    byte 0 -> Left(1), byte 1 -> Right(2), byte 2 -> Attack(4), non-zero = pressed.
    """
    a = np.asarray(actions)
    if a.ndim == 2:
        if a.shape[1] != 3:
            raise ValueError("actions must be (N,3) booleans or (N,) ints, got shape %s" % (a.shape,))
        a = a != 0
        return (a[:, 0].astype(np.uint8) | (a[:, 1].astype(np.uint8) << 1) | (a[:, 2].astype(np.uint8) << 2))
    if a.ndim == 1:
        if a.size and (a.min() < 0 or a.max() > 7):
            raise ValueError("integer actions must be in 0..7")
        return a.astype(np.uint8)
    raise ValueError("actions must be (N,3) booleans or (N,) ints, got shape %s" % (a.shape,))


def decode_actions(bits):
    """uint8 3-bit inputs -> (N,3) booleans (FootsiesState.__post_init__, state.py:26-36).  Three
    bit tests stacked: a (256, 3) table gathered with the codes measured 5x slower in numpy."""
    b = np.asarray(bits, dtype=np.uint8)
    return np.stack([(b & 1) != 0, (b & 2) != 0, (b & 4) != 0], axis=-1)


class FootsiesSim:
    """N independent FOOTSIES arenas on one MI355X.

    Parameters mirror ``fs_config`` (include/footsies.h).  ``outputs()`` returns
    torch tensors on the device that are overwritten by the next call.
    """

    def __init__(self, num_envs, device=0, p2_mode="bot", dense_reward=True, float_mode="strict",
                 autoreset_mode="same_step", seed=0, frame_delay=0, p1_mode="external", arena_base=0,
                 host_outputs=False, backend=None):
        if backend not in (None, "torch", "native"):
            raise ValueError("backend must be 'torch' or 'native'")
        torch = _torch_or_none() if backend != "native" else None
        if backend == "torch" and torch is None:
            raise ImportError("FootsiesSim(backend='torch') needs PyTorch")
        if torch is None and not host_outputs:
            raise ImportError("FootsiesSim with device outputs needs PyTorch; without it use host_outputs=True "
                              "(the numpy FootsiesVectorEnv / FootsiesEnv do)")
        self._native = torch is None
        if not self._native and not torch.cuda.is_available():
            raise RuntimeError("FootsiesSim needs a HIP device (torch.cuda.is_available() is False)")
        if p2_mode not in P2_MODES:
            raise ValueError("p2_mode must be one of %s" % list(P2_MODES))
        if float_mode not in FLOAT_MODES:
            raise ValueError("float_mode must be one of %s" % list(FLOAT_MODES))
        if autoreset_mode not in AUTORESET_MODES:
            raise ValueError("autoreset_mode must be one of %s" % list(AUTORESET_MODES))
        if p1_mode not in P1_MODES:
            raise ValueError("p1_mode must be one of %s" % list(P1_MODES))
        self.num_envs = int(num_envs)
        self.device = int(device) if self._native else torch.device("cuda", device)
        self._dev_index = int(device) if self._native else self.device.index
        self._host_mem = None
        self.p2_mode = p2_mode
        self.p1_mode = p1_mode
        self.autoreset_mode = autoreset_mode
        cfg = _abi.fs_config(num_envs=self.num_envs, device_id=device, p2_mode=P2_MODES[p2_mode],
                             dense_reward=int(bool(dense_reward)), frame_delay=int(frame_delay),
                             float_mode=FLOAT_MODES[float_mode], autoreset_mode=AUTORESET_MODES[autoreset_mode],
                             base_seed=int(seed) & 0xFFFFFFFFFFFFFFFF, p1_mode=P1_MODES[p1_mode],
                             arena_base=int(arena_base))
        h = C.c_void_p()
        check(lib().fs_create(C.byref(cfg), C.byref(h)), None)
        self._h = h
        self.cfg = cfg
        # outputs: torch tensors bound into the library, all views of one device buffer (256-B
        # aligned slices) so that the host side fetches a step's outputs with one copy
        n = self.num_envs
        self._out = {}
        layout, total = [], 0
        for name, (dt, cols) in _abi.OUTPUT_SPEC.items():
            shape = (n, cols) if cols > 1 else (n,)
            nbytes = n * cols * np.dtype(dt).itemsize
            layout.append((name, dt, shape, total, nbytes))
            total += (nbytes + 255) // 256 * 256
        # host_outputs: the bound buffers are pinned host memory, which the kernels write across
        # the bus; a step's outputs are then on the host once the stream is done, with no copy
        # (the single-arena drop-in, where the copy's own latency was a third of a step).
        # outputs() then returns host tensors; every call that returns them (step, reset, step_n
        # without a trajectory, outputs) first waits for the handle's stream, so they never hold
        # an earlier tick's values while the kernels are still writing (_host_ready).
        # (the pinned host buffer comes from the library, fs_host_alloc, which also gives its device
        # address: no second HIP runtime is ever loaded by name from here)
        self.host_outputs = bool(host_outputs)
        if self.host_outputs:
            hp, dp = C.c_void_p(), C.c_void_p()
            rc = lib().fs_host_alloc(self._dev_index, total, C.byref(hp), C.byref(dp))
            if rc:
                lib().fs_destroy(h)
                self._h = None
                check(rc, None)
            self._host_mem = _HostBuffer(hp.value)
            raw = (C.c_uint8 * total).from_address(hp.value)
            raw._owner = self._host_mem  # every view of the buffer keeps it allocated (freed with the last)
            host = np.frombuffer(raw, dtype=np.uint8)
            self._out_buf = host if self._native else torch.from_numpy(host)
            base, host_base = dp.value, hp.value
        else:
            with torch.cuda.device(self.device):
                self._out_buf = torch.zeros(total, dtype=torch.uint8, device=self.device)
            base = host_base = self._out_buf.data_ptr()
        for name, dt, shape, off, nbytes in layout:
            if self._native:
                self._out[name] = self._out_buf[off:off + nbytes].view(dt).reshape(shape)
            else:
                self._out[name] = self._out_buf[off:off + nbytes].view(getattr(torch, _TORCH_DTYPES[dt])).view(shape)
        self._out_layout = layout
        self._host_buf = None  # pinned mirror of _out_buf, allocated on first use
        # the library's creation-time outputs (state(-1)) into the bound buffers
        own = _abi.fs_outputs()
        check(lib().fs_outputs_get(h, C.byref(own)), h)
        check(lib().fs_sync(h), h)
        for name, dt, shape, off, nbytes in layout:
            check(lib().fs_memcpy(C.c_void_p(host_base + off), C.c_void_p(getattr(own, name)), nbytes), None)
        bind = _abi.fs_outputs(**{name: base + off for name, _, _, off, _ in layout})
        check(lib().fs_bind_outputs(h, C.byref(bind)), h)
        if self._native:
            self._stream = None  # the library's own stream
        else:
            self.use_torch_stream()

    # -- streams ---------------------------------------------------------------------
    def use_torch_stream(self, stream=None):
        """Issue all further work on ``stream`` (default: torch's current stream)."""
        self._need_torch("use_torch_stream")
        torch = _torch()
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        check(lib().fs_set_stream(self._h, C.c_void_p(s.cuda_stream)), self._h)
        self._stream = s

    def _need_torch(self, what):
        if self._native:
            raise RuntimeError("FootsiesSim.%s needs PyTorch (this handle runs without it: backend='native')" % what)

    @property
    def backend(self):
        return "native" if self._native else "torch"

    @property
    def stream(self):
        """The torch stream the library issues this handle's kernels on (use_torch_stream)."""
        return self._stream

    # -- core API --------------------------------------------------------------------
    def reset(self, seeds=None, mask=None, hard=False, seed_only=False):
        """FootsiesEnv.reset over all (or the masked) arenas; seeds -> Random.InitState.
        seed_only: the SEED command alone (no reset, outputs untouched)."""
        n = self.num_envs
        s = None if seeds is None else np.ascontiguousarray(np.broadcast_to(np.asarray(seeds, dtype=np.uint64), (n,)))
        m = None if mask is None else np.ascontiguousarray(np.asarray(mask, dtype=np.uint8).reshape(n))
        flags = _abi.FS_RESET_SEED_ONLY if seed_only else (_abi.FS_RESET_HARD if hard else _abi.FS_RESET_IF_NEEDED)
        check(lib().fs_reset(self._h, None if s is None else s.ctypes.data, None if m is None else m.ctypes.data,
                             flags), self._h)
        return self._ready_out()

    def set_p2_mode(self, mode, mask=None):
        """P2 of the masked arenas (all by default) becomes the in-game bot (mode "bot") or the
        remote actor again ("external"): the P2_BOT command (fs_set_p2_mode).  Only for a sim
        created with p2_mode="external"."""
        if mode not in ("external", "bot"):
            raise ValueError("mode must be 'external' or 'bot'")
        m = None if mask is None else np.ascontiguousarray(np.asarray(mask, dtype=np.uint8).reshape(self.num_envs))
        check(lib().fs_set_p2_mode(self._h, P2_MODES[mode], None if m is None else m.ctypes.data), self._h)

    def step(self, p1, p2=None, active=None):
        """One env-step of every arena.  Actions: torch uint8 device tensors [N] (fast path) or
        host arrays ((N,3) bools or (N,) ints).  active: optional [N] mask -- only those arenas
        tick (fs_step_masked); the others keep their state and outputs.  With p1_mode="bot"
        (by_example) p1 is ignored and may be None."""
        ext = self.p2_mode == "external"
        if self._native:  # host arrays only
            if ext and p2 is None:
                raise ValueError("p2 actions are required when p2_mode='external'")
            if p1 is None:
                if self.p1_mode != "bot":
                    raise ValueError("p1 actions are required unless p1_mode='bot'")
                p1 = np.zeros(self.num_envs, np.uint8)
            return self._step_host(p1, p2 if ext else None, active)
        torch = _torch()
        # the RL loop's case first: uint8 [N] contiguous tensors on this handle's GPU, no mask
        # (the ctypes prototype takes the raw pointers as ints; nothing is converted or copied)
        if active is None and _fast_actions(p1, self._dev_index, self.num_envs) and (
                _fast_actions(p2, self._dev_index, self.num_envs) if ext else p2 is None):
            rc = lib().fs_step(self._h, p1.data_ptr(), p2.data_ptr() if ext else None, _abi.FS_ACT_DEVICE)
            if rc:
                check(rc, self._h)
            return self._ready_out()
        if ext and p2 is None:
            raise ValueError("p2 actions are required when p2_mode='external'")
        if p1 is None:
            if self.p1_mode != "bot":
                raise ValueError("p1 actions are required unless p1_mode='bot'")
            p1 = np.zeros(self.num_envs, np.uint8) if not any(
                isinstance(x, torch.Tensor) and x.is_cuda for x in (p2, active)) else torch.zeros(
                    self.num_envs, dtype=torch.uint8, device=self.device)
        on_device = any(isinstance(x, torch.Tensor) and x.is_cuda for x in (p1, p2, active))
        if on_device:  # device path: anything on the host is moved over first
            p1 = _as_u8_device(_to_device(p1, self.device), self.num_envs)
            p2t = _as_u8_device(_to_device(p2, self.device), self.num_envs) if ext else None
            q2 = C.c_void_p(p2t.data_ptr()) if ext else None
            if active is None:
                check(lib().fs_step(self._h, C.c_void_p(p1.data_ptr()), q2, _abi.FS_ACT_DEVICE), self._h)
            else:
                m = torch.as_tensor(active, device=self.device).reshape(self.num_envs).to(torch.uint8).contiguous()
                check(lib().fs_step_masked(self._h, C.c_void_p(p1.data_ptr()), q2, C.c_void_p(m.data_ptr()),
                                           _abi.FS_ACT_DEVICE), self._h)
        else:
            return self._step_host(p1, p2 if ext else None, active)
        return self._ready_out()

    def _step_host(self, p1, p2, active):
        """fs_step / fs_step_masked with host actions (FS_ACT_HOST: the library stages them)."""
        a1 = np.ascontiguousarray(encode_actions(_host(p1)))
        a2 = np.ascontiguousarray(encode_actions(_host(p2))) if p2 is not None else None
        if a1.shape[0] != self.num_envs or (a2 is not None and a2.shape[0] != self.num_envs):
            raise ValueError("expected %d actions" % self.num_envs)
        q2 = None if a2 is None else a2.ctypes.data
        if active is None:
            check(lib().fs_step(self._h, a1.ctypes.data, q2, _abi.FS_ACT_HOST), self._h)
        else:
            m = np.ascontiguousarray(np.asarray(active).reshape(self.num_envs), dtype=np.uint8)
            check(lib().fs_step_masked(self._h, a1.ctypes.data, q2, m.ctypes.data, _abi.FS_ACT_HOST), self._h)
        return self._ready_out()

    def _check_device(self, t, name, dtype, numel):
        """A buffer the kernels read or write through its raw pointer: a contiguous torch tensor of
        `dtype` on this handle's GPU with at least `numel` elements (anything else would hand the
        kernel a host or foreign-device address, or let it run past the end)."""
        self._need_torch("_check_device")
        torch = _torch()
        if not (isinstance(t, torch.Tensor) and t.is_cuda and t.get_device() == self._dev_index and t.dtype == dtype
                and t.is_contiguous() and t.numel() >= numel):
            raise ValueError("%s: a contiguous %s tensor on %s with >= %d elements is required" % (
                name, dtype, self.device, numel))

    def step_n(self, n, p1=None, p2=None, action_seed=0, trajectory=None):
        """n ticks in one kernel launch.  p1/p2: device uint8 [n][N] or None (on-device hashed
        actions).  trajectory: dict of device tensors shaped [n][N](,2) like ``alloc_trajectory``."""
        self._need_torch("step_n")
        torch = _torch()
        n = int(n)
        for name, a in (("p1", p1), ("p2", p2)):
            if a is not None:
                self._check_device(a, name, torch.uint8, n * self.num_envs)
        t = None
        if trajectory is not None:
            for k in _abi.OUTPUT_SPEC:
                if k in trajectory:
                    dt, cols = _abi.OUTPUT_SPEC[k]
                    self._check_device(trajectory[k], "trajectory[%r]" % k, getattr(torch, _TORCH_DTYPES[dt]),
                                       n * self.num_envs * cols)
            t = _abi.fs_outputs(**{k: trajectory[k].data_ptr() for k in _abi.OUTPUT_SPEC if k in trajectory})
        check(lib().fs_step_n(self._h, int(n), None if p1 is None else C.c_void_p(p1.data_ptr()),
                              None if p2 is None else C.c_void_p(p2.data_ptr()), int(action_seed) & (2**64 - 1),
                              None if t is None else C.byref(t)), self._h)
        return trajectory if trajectory is not None else self._ready_out()

    def hash_actions(self, n_steps, seed=0x5EED, t0=0, p2=True):
        """Device uint8 [n_steps][N] action arrays from the synthetic splitmix64 stream."""
        self._need_torch("hash_actions")
        torch = _torch()
        p1 = torch.empty((n_steps, self.num_envs), dtype=torch.uint8, device=self.device)
        q2 = torch.empty((n_steps, self.num_envs), dtype=torch.uint8, device=self.device) if p2 else None
        check(lib().fs_hash_actions(self._h, int(n_steps), int(seed), int(t0), C.c_void_p(p1.data_ptr()),
                                    C.c_void_p(q2.data_ptr()) if p2 else None), self._h)
        return p1, q2

    def alloc_packed_trajectory(self, n):
        """Device buffers for step_n_packed: {"lanes": uint8 [n][N][2][16], "reward": float64
        [n][N], "final_lanes": uint8 [n][N][2][16] (same-step auto-reset only, else None)}
        (include/footsies.h fs_packed_traj); unpack_trajectory gives their per-field views."""
        self._need_torch("alloc_packed_trajectory")
        torch = _torch()
        shape = (n, self.num_envs, 2, _abi.FS_PACKED_LANE_BYTES)
        same = self.autoreset_mode == "same_step"
        return {"lanes": torch.zeros(shape, dtype=torch.uint8, device=self.device),
                "reward": torch.zeros((n, self.num_envs), dtype=torch.float64, device=self.device),
                "final_lanes": torch.zeros(shape, dtype=torch.uint8, device=self.device) if same else None}

    def step_n_packed(self, n, p1, p2=None, trajectory=None):
        """step_n with device action rows p1 / p2 (uint8 [n][N]) into a packed trajectory
        (fs_step_n_packed: two stores per tick instead of ten; alloc_packed_trajectory)."""
        self._need_torch("step_n_packed")
        torch = _torch()
        n = int(n)
        traj = trajectory if trajectory is not None else self.alloc_packed_trajectory(n)
        rows = n * self.num_envs
        self._check_device(p1, "p1", torch.uint8, rows)
        if p2 is not None:
            self._check_device(p2, "p2", torch.uint8, rows)
        self._check_device(traj["lanes"], "lanes", torch.uint8, rows * 2 * _abi.FS_PACKED_LANE_BYTES)
        self._check_device(traj["reward"], "reward", torch.float64, rows)
        fl = traj.get("final_lanes")
        if fl is not None:
            self._check_device(fl, "final_lanes", torch.uint8, rows * 2 * _abi.FS_PACKED_LANE_BYTES)
        t = _abi.fs_packed_traj(lanes=traj["lanes"].data_ptr(), reward=traj["reward"].data_ptr(),
                                final_lanes=None if fl is None else fl.data_ptr())
        check(lib().fs_step_n_packed(self._h, int(n), C.c_void_p(p1.data_ptr()),
                                     None if p2 is None else C.c_void_p(p2.data_ptr()), C.byref(t)), self._h)
        return traj

    def alloc_trajectory(self, n):
        self._need_torch("alloc_trajectory")
        torch = _torch()
        out = {}
        for name, (dt, cols) in _abi.OUTPUT_SPEC.items():
            shape = (n, self.num_envs, cols) if cols > 1 else (n, self.num_envs)
            out[name] = torch.zeros(shape, dtype=getattr(torch, _TORCH_DTYPES[dt]), device=self.device)
        return out

    def outputs(self):
        return self._ready_out()

    def _ready_out(self):
        """The bound outputs, safe to read: with host_outputs the kernels write them into pinned
        host memory asynchronously, so the handle's stream is waited for first (device tensors are
        ordered by the stream and need no wait)."""
        if self.host_outputs:
            check(lib().fs_sync(self._h), self._h)
        return self._out

    def step_records(self, p1, p2=None, dst=None):
        """step() of every arena that also writes the step's 40-byte records (fs_step_rec: the
        bytes pack_outputs would, from the tick's own kernel); device uint8 [N] actions (p1 may
        be None with p1_mode="bot").  Returns the [N, 40] uint8 device records."""
        self._need_torch("step_records")
        torch = _torch()
        if dst is None:
            dst = torch.empty((self.num_envs, _abi.FS_RECORD_BYTES), dtype=torch.uint8, device=self.device)
        self._check_device(dst, "dst", torch.uint8, self.num_envs * _abi.FS_RECORD_BYTES)
        ext = self.p2_mode == "external"
        q1 = None if p1 is None else _as_u8_device(_to_device(p1, self.device), self.num_envs)
        q2 = _as_u8_device(_to_device(p2, self.device), self.num_envs) if ext else None
        if q1 is None and self.p1_mode != "bot":
            raise ValueError("p1 actions are required unless p1_mode='bot'")
        check(lib().fs_step_rec(self._h, None if q1 is None else C.c_void_p(q1.data_ptr()),
                                None if q2 is None else C.c_void_p(q2.data_ptr()), _abi.FS_ACT_DEVICE,
                                C.c_void_p(dst.data_ptr())), self._h)
        self._ready_out()
        return dst

    def pack_outputs(self, dst=None):
        """The current outputs as one 40-byte record per arena ([N, 40] uint8 device tensor,
        parallel.RECORD_BYTES layout) by one kernel (fs_pack_outputs): the gather payload."""
        self._need_torch("pack_outputs")
        torch = _torch()
        if dst is None:
            dst = torch.empty((self.num_envs, _abi.FS_RECORD_BYTES), dtype=torch.uint8, device=self.device)
        check(lib().fs_pack_outputs(self._h, C.c_void_p(dst.data_ptr())), self._h)
        return dst

    def outputs_numpy(self, copy=True, _synced=False):
        """The current outputs on the host, fetched with one device-to-host copy into a pinned
        buffer.  copy=False returns views of that buffer, overwritten by the next call.
        (_synced, internal: with host_outputs, the caller has just waited for the stream --
        step / reset returned -- and nothing was issued since.)"""
        if self._host_buf is None:
            self._host_buf = (self._out_buf if self.host_outputs else
                              _torch().empty(self._out_buf.numel(), dtype=_torch().uint8, pin_memory=True))
            host = self._host_buf if self._native else self._host_buf.numpy()
            # the typed views of the pinned buffer, made once (building them costs ~20 us a call)
            self._host_views = {name: host[off:off + nbytes].view(dt).reshape(shape)
                                for name, dt, shape, off, nbytes in self._out_layout}
        if self.host_outputs:  # the kernels wrote them there: wait for the handle's stream
            if not _synced:
                check(lib().fs_sync(self._h), self._h)
        else:
            # on the handle's own stream, so the copy is ordered after the library's kernels whatever
            # torch's current stream is (a blocking copy: it returns once the bytes are on the host)
            torch = _torch()
            with torch.cuda.stream(self._stream):
                self._host_buf.copy_(self._out_buf)
        if copy:
            return {name: v.copy() for name, v in self._host_views.items()}
        return dict(self._host_views)

    def env_state(self):
        arr = (_abi.fs_env_state * self.num_envs)()
        check(lib().fs_get_env_state(self._h, arr), self._h)
        return np.ctypeslib.as_array(arr).copy()

    def get_state(self):
        arr = (_abi.fs_arena_state * self.num_envs)()
        check(lib().fs_get_state(self._h, arr), self._h)
        return np.ctypeslib.as_array(arr).copy()

    def set_state(self, state):
        state = np.ascontiguousarray(state)
        if state.shape != (self.num_envs,):
            raise ValueError("state must have shape (%d,)" % self.num_envs)
        arr = (_abi.fs_arena_state * self.num_envs).from_buffer_copy(state.tobytes())
        check(lib().fs_set_state(self._h, arr), self._h)

    def sync(self):
        check(lib().fs_sync(self._h), self._h)

    @property
    def handle(self):
        return self._h

    @property
    def steps_taken(self):
        return int(lib().fs_steps_taken(self._h))

    def close(self):
        if getattr(self, "_h", None):
            lib().fs_sync(self._h)
            lib().fs_destroy(self._h)
            self._h = None
        if getattr(self, "_host_mem", None):
            # (the pinned buffer is freed when its last view is gone: outputs_numpy(copy=False) views
            # a caller still holds stay readable, no longer written)
            self._out = {}
            self._host_views = {}
            self._out_buf = self._host_buf = None
            self._host_mem = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _HostBuffer:
    """Pinned host memory from fs_host_alloc, released by fs_host_free when the last numpy / torch
    view of it goes away."""

    def __init__(self, ptr):
        self.ptr = ptr

    def __del__(self):
        try:
            lib().fs_host_free(C.c_void_p(self.ptr))
        except Exception:  # (interpreter shutdown)
            pass


def _host(a):
    torch = _torch_or_none()
    if torch is not None and isinstance(a, torch.Tensor):
        return a.detach().cpu().numpy()
    return a


def unpack_trajectory(traj):
    """The per-field views (alloc_trajectory's names, dtypes and shapes) of a packed trajectory
    (FootsiesSim.alloc_packed_trajectory; torch tensors or numpy arrays): strided views, no copy.
    final_* appear when the trajectory has final_lanes."""
    is_np = isinstance(traj["lanes"], np.ndarray)

    def typed(buf, kind):  # the 16-B records as 4 words of one type
        if is_np:
            return buf.view({"u8": np.uint8, "f32": np.float32, "i32": np.int32}[kind])
        torch = _torch()
        return buf.view({"u8": torch.uint8, "f32": torch.float32, "i32": torch.int32}[kind])

    out = {}
    for pre, key in (("", "lanes"), ("final_", "final_lanes")):
        buf = traj.get(key)
        if buf is None:
            continue
        b, f, i = typed(buf, "u8"), typed(buf, "f32"), typed(buf, "i32")
        out[pre + "guard"], out[pre + "move"] = b[..., 0], b[..., 1]
        out[pre + "action"], out[pre + "hitstun"] = b[..., 2], b[..., 3]
        out[pre + "move_frame"], out[pre + "position"] = f[..., 1], f[..., 2]
        out[pre + "frame"] = i[..., 0, 3]
        if not pre:
            out["terminated"], out["truncated"] = b[..., 1, 12], b[..., 1, 13]
    out["reward"] = traj["reward"]
    return out


def _fast_actions(t, dev_index, n):
    """Device actions that fs_step can take as they are: a contiguous uint8 [n] CUDA tensor on the
    handle's device."""
    torch = _torch()
    return (type(t) is torch.Tensor and t.dtype is torch.uint8 and t.is_cuda and t.get_device() == dev_index
            and t.dim() == 1 and t.shape[0] == n and t.is_contiguous())


def _to_device(a, device):
    torch = _torch()
    if isinstance(a, torch.Tensor):
        return a.to(device)
    return torch.as_tensor(encode_actions(np.asarray(a)), device=device)


def _as_u8_device(t, n):
    torch = _torch()
    if t.dim() == 2 and t.shape[1] == 3:
        t = t.to(torch.uint8)
        t = t[:, 0] | (t[:, 1] << 1) | (t[:, 2] << 2)
    if t.dtype != torch.uint8:
        t = t.to(torch.uint8)
    t = t.contiguous()
    if t.shape != (n,):
        raise ValueError("expected device actions of shape (%d,), got %s" % (n, tuple(t.shape)))
    return t

