"""On-device rollouts with a policy in the loop.

Every step: the simulator's outputs (device tensors, written in place by libfootsies.so)
-> features -> a 2x64 MLP actor -> a sampled action per arena (Gumbel-max over Exp(1) noise,
with its log-probability for PPO) -> fs_step with device actions.  Nothing leaves the GPU and
nothing synchronises, so a block of steps is captured once into a HIP graph and
replayed: the loop then costs graph launches, not the ~20 kernel launches per step.

Graph replays do not advance the handle's host-side step counter (fs_steps_taken), which
only the hashed-action stream and frame_delay > 0 read; use eager steps for those.

:class:`FusedPolicyRollout` goes one step further: the actor runs inside the simulator's
fused tick loop (fs_step_n_policy, csrc/fs_policy.h) as bf16 MFMAs, so a block of n
policy-driven ticks is one kernel launch with the arena state in registers throughout.
"""
import ctypes as C

from . import _abi
from ._lib import check, lib

N_FEATURES = 8
N_ACTIONS = 8  # (left, right, attack) combinations, FootsiesActionCombinationsDiscretized


def _torch():
    import torch
    return torch


def obs_features(out):
    """[N, 8] float32: guard / 3, move / 16, move_frame / 55, position / 4.6 for P1 and P2
    (the reference's normalisation constants, wrappers/normalization.py)."""
    torch = _torch()
    return torch.cat([out["guard"].float() / 3.0, out["move"].float() / 16.0, out["move_frame"] / 55.0,
                      out["position"] / 4.6], dim=1)


def make_actor(hidden=64, device=None, seed=0):
    """The C5 actor: Linear(8, 64) - tanh - Linear(64, 64) - tanh - Linear(64, 8), random init."""
    torch = _torch()
    g = torch.Generator().manual_seed(seed)
    nn = torch.nn
    net = nn.Sequential(nn.Linear(N_FEATURES, hidden), nn.Tanh(), nn.Linear(hidden, hidden), nn.Tanh(),
                        nn.Linear(hidden, N_ACTIONS))
    with torch.no_grad():
        for p in net.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.3)
    return net.to(device)


class PolicyRollout:
    """Steps `sim` (a FootsiesSim) with actions sampled from `actor`; P2 is whatever the
    handle was created with (bot, noop, or `p2_actions` for external)."""

    def __init__(self, sim, actor, p2_actions=None):
        torch = _torch()
        self.sim, self.actor = sim, actor
        n = sim.num_envs
        dev = sim.device
        self.action = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.logp = torch.zeros(n, dtype=torch.float32, device=dev)
        # obs_features' divisors per column: one cat + one division gives its values bit for bit
        self._div = torch.tensor([3.0, 3.0, 16.0, 16.0, 55.0, 55.0, 4.6, 4.6], dtype=torch.float32, device=dev)
        self.p2 = p2_actions if p2_actions is not None else torch.zeros(n, dtype=torch.uint8, device=dev)
        self.graph = None
        self.graph_steps = 0
        self.action_log = None  # [graph steps][N] actions of the last replay when capture(log=True)

    def _step(self, log_row=None):
        torch = _torch()
        out = self.sim.outputs()
        with torch.no_grad():  # (17 kernels per step with fs_step: each one is a graph node)
            x = torch.cat([out["guard"].float(), out["move"].float(), out["move_frame"], out["position"]], dim=1)
            logits = self.actor(x.div_(self._div))  # == obs_features(out)
            # Gumbel-max with -log(-log U) = -log E, E ~ Exp(1)
            a = torch.argmax(logits - torch.empty_like(logits).exponential_().log_(), dim=1)
            torch.gather(torch.log_softmax(logits, dim=1), 1, a[:, None], out=self.logp.view(-1, 1))
            self.action.copy_(a)
            if log_row is not None:
                log_row.copy_(self.action)
        check(lib().fs_step(self.sim.handle, C.c_void_p(self.action.data_ptr()), C.c_void_p(self.p2.data_ptr()),
                            _abi.FS_ACT_DEVICE), self.sim.handle)

    def step_eager(self, n=1):
        for _ in range(n):
            self._step()

    def capture(self, steps, warmup=2, log=False):
        """Capture `steps` policy+simulator steps into one HIP graph on a private stream, after
        `warmup` eager steps there (library / BLAS handles and the allocator settle outside the
        capture).  Returns the warm-up steps' actions ([warmup][N], host) so they can be replayed."""
        torch = _torch()
        stream = torch.cuda.Stream(device=self.sim.device)
        self.sim.use_torch_stream(stream)  # the library issues its kernels on the capture stream
        warm = []
        with torch.cuda.stream(stream):
            for _ in range(warmup):
                self._step()
                warm.append(self.action.cpu())
        stream.synchronize()
        if log:
            self.action_log = torch.zeros((steps, self.sim.num_envs), dtype=torch.uint8, device=self.sim.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for i in range(steps):
                self._step(self.action_log[i] if log else None)
        self.graph, self.graph_steps, self.stream = g, steps, stream
        return warm

    def replay(self, times=1):
        for _ in range(times):
            self.graph.replay()


class FusedPolicyRollout:
    """C5 in one launch per block of ticks: `actor` (the make_actor shape, 8-64-64-8 with tanh)
    is evaluated in bf16 inside the simulator kernel, P1's action drawn from its softmax by
    inverse CDF with a counter-based uniform of (seed, env, step).  P2 is whatever the handle
    was created with (bot, noop, or `p2_actions` [n][N] per call for external)."""

    def __init__(self, sim, actor, seed=0):
        torch = _torch()
        lin = [m for m in actor if isinstance(m, torch.nn.Linear)]
        shapes = [tuple(m.weight.shape) for m in lin]
        if shapes != [(64, N_FEATURES), (64, 64), (N_ACTIONS, 64)]:
            raise ValueError("the fused actor is 8 -> 64 -> 64 -> 8; got %s" % (shapes,))
        self.sim, self.seed = sim, int(seed) & (2**64 - 1)
        with torch.no_grad():
            self.params = [t.detach().to(device=sim.device, dtype=torch.float32).contiguous()
                           for m in lin for t in (m.weight, m.bias)]

    def refresh(self, actor):
        """Copy new actor weights in (after an optimiser step); the buffers stay put."""
        torch = _torch()
        lin = [m for m in actor if isinstance(m, torch.nn.Linear)]
        with torch.no_grad():
            for dst, src in zip(self.params, [t for m in lin for t in (m.weight, m.bias)]):
                dst.copy_(src)

    def rollout(self, n, actions=None, logp=None, p2_actions=None, trajectory=None):
        """n policy-driven ticks in one launch.  `actions` (uint8) / `logp` (float32) [n][N]
        device tensors receive P1's samples (allocated when None; pass False to skip one).
        Returns (actions, logp)."""
        torch = _torch()
        N, dev = self.sim.num_envs, self.sim.device
        if actions is None:
            actions = torch.empty((n, N), dtype=torch.uint8, device=dev)
        if logp is None:
            logp = torch.empty((n, N), dtype=torch.float32, device=dev)
        w = self.params
        pol = _abi.fs_policy(w1=w[0].data_ptr(), b1=w[1].data_ptr(), w2=w[2].data_ptr(), b2=w[3].data_ptr(),
                             w3=w[4].data_ptr(), b3=w[5].data_ptr(), seed=self.seed,
                             actions_out=actions.data_ptr() if actions is not False else None,
                             logp_out=logp.data_ptr() if logp is not False else None)
        t = None
        if trajectory is not None:
            t = _abi.fs_outputs(**{k: trajectory[k].data_ptr() for k in _abi.OUTPUT_SPEC if k in trajectory})
        check(lib().fs_step_n_policy(self.sim.handle, int(n), C.byref(pol),
                                     None if p2_actions is None else C.c_void_p(p2_actions.data_ptr()),
                                     None if t is None else C.byref(t)), self.sim.handle)
        return actions, logp
