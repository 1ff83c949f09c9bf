"""A small PPO learner over fused rollouts (BASELINE config C5: "65 536 envs driving a small
PPO actor (PyTorch-ROCm), end-to-end steps/sec with policy in the loop").

One iteration:
1. `horizon` policy-driven ticks of every arena in one kernel launch (fs_step_n_policy).
   P1's actions are sampled by the bf16 actor inside the tick loop, and every tick's
   outputs land in a [horizon][N] trajectory in HBM.
2. Features of the horizon + 1 observations, critic values, and GAE advantages, in torch on
   the same device. The observation before tick t is the output of tick t - 1 (after a
   same-step auto-reset that is the fresh round's state, so a terminal tick's successor is
   never bootstrapped through: done masks it).
3. `epochs` x `minibatches` clipped-surrogate updates of the actor and critic (fp32 Adam; the
   gradients' 64x64 hidden layer on split-bf16 MFMAs by default since round 4,
   `learner_precision="fp32"` for fp32 FMAs).  With
   `learner="hip"` (the default) each minibatch's loss and gradient come from one fused
   forward + backward kernel per network (fs_ppo_grad, csrc/fs_learn.hip) straight into the
   parameters' .grad; `learner="torch"` runs the same loss through torch autograd (the
   definition the kernel is tested against, tests/test_gpu_learn.py).  Adam is torch's.
   The importance ratio's old log-probabilities are the behaviour policy's: the log-probs the
   bf16 kernel actor sampled with (`old_logp="behaviour"`, the default), or the same network
   recomputed in fp32 (`old_logp="fp32"`, first ratio exactly 1).  Either way the iteration
   reports how far the two are apart: `kl_behaviour_fp32`, the sample estimate
   E_a~behaviour[log p_bf16(a) - log p_fp32(a)] of KL(bf16 actor || fp32 actor), and
   `logp_abs_diff`, the mean |log p_bf16(a) - log p_fp32(a)|.  The fp32 log-probs come from
   fs_ppo_eval at fp32 FMAs (FS_PPO_FP32) whatever the learner's precision; the critic values and
   the gradients use `learner_precision`, whatever `old_logp` is (`PPOTrainer.prepare`).
4. The new actor weights are copied into the rollout's device buffers (no reallocation).

Nothing leaves the GPU inside an iteration, and the simulator never waits on the host.
"""
import ctypes as C
import time

from . import _abi
from ._lib import check, lib
from .rollout import N_ACTIONS, N_FEATURES, FusedPolicyRollout, make_actor, obs_features


def _torch():
    import torch
    return torch


def make_critic(hidden=64, device=None, seed=1):
    torch = _torch()
    g = torch.Generator().manual_seed(seed)
    nn = torch.nn
    net = nn.Sequential(nn.Linear(N_FEATURES, hidden), nn.Tanh(), nn.Linear(hidden, hidden), nn.Tanh(),
                        nn.Linear(hidden, 1))
    with torch.no_grad():
        for p in net.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.1)
    return net.to(device)


_WGRAD_CHUNK = 8192
_SHUFFLE_CHUNK = 2048  # minibatches are drawn as shuffled runs of this many consecutive samples


def _weight_grad(g, x):
    """g^T x for tall, skinny g [M, out] and x [M, in] (M ~ 2M samples, out/in <= 64): one
    batched GEMM over row chunks, then a sum over the chunks.  A single GEMM with a reduction
    dimension of millions and a 64 x 64 result leaves hipBLASLt a handful of output tiles to
    split; the batched form runs ~13x faster on MI355X (fp32, 2.1M x 64: 0.2 ms vs 2.6 ms)."""
    torch = _torch()
    M = g.shape[0]
    full = (M // _WGRAD_CHUNK) * _WGRAD_CHUNK
    out = torch.zeros((g.shape[1], x.shape[1]), dtype=g.dtype, device=g.device)
    if full:
        gc = g[:full].reshape(-1, _WGRAD_CHUNK, g.shape[1])
        xc = x[:full].reshape(-1, _WGRAD_CHUNK, x.shape[1])
        out += torch.bmm(gc.transpose(1, 2), xc).sum(0)
    if full < M:
        out += g[full:].t() @ x[full:]
    return out


def _linear_fn():
    torch = _torch()

    class SkinnyLinear(torch.autograd.Function):
        """y = x W^T + b with the weight gradient formed by `_weight_grad`."""

        @staticmethod
        def forward(ctx, x, w, b):
            ctx.save_for_backward(x, w)
            return torch.addmm(b, x, w.t())

        @staticmethod
        def backward(ctx, gy):
            x, w = ctx.saved_tensors
            gy = gy.contiguous()
            gx = gy @ w if ctx.needs_input_grad[0] else None  # (the first layer's input is data)
            return gx, _weight_grad(gy, x.contiguous()), gy.sum(0)

    return SkinnyLinear


_SKINNY = None


def mlp(net, x):
    """net(x) for an nn.Sequential of Linear / activation layers, with every Linear through
    SkinnyLinear (same values; the weight gradients take the batched path)."""
    global _SKINNY
    torch = _torch()
    if _SKINNY is None:
        _SKINNY = _linear_fn()
    for m in net:
        x = _SKINNY.apply(x, m.weight, m.bias) if isinstance(m, torch.nn.Linear) else m(x)
    return x


class PPOGrad:
    """fs_ppo_grad for an actor (8-64-64-8) and a critic (8-64-64-1): each call writes the
    minibatch gradient of PPO's loss into one flat device buffer whose views are the
    parameters' ``.grad`` (set once here), and returns the device [3] of (policy, value,
    entropy) loss means.

    precision: "fp32" (default) runs the 64x64 hidden layer on fp32 FMAs; "split_bf16"
    (FS_PPO_SPLIT_BF16) runs it on bf16 MFMAs with each fp32 operand split into a bf16 high
    and low part (hi*hi + hi*lo + lo*hi, fp32 accumulation: ~2^-16 relative per product) --
    same results to ~1e-5 relative, not bit-identical to the fp32 path."""

    PRECISIONS = {"fp32": _abi.FS_PPO_FP32, "split_bf16": _abi.FS_PPO_SPLIT_BF16}

    def __init__(self, actor, critic, precision="fp32"):
        torch = _torch()
        if precision not in self.PRECISIONS:
            raise ValueError("precision must be one of %s" % sorted(self.PRECISIONS))
        self.precision = precision
        self._prec = self.PRECISIONS[precision]
        self._modules = (actor, critic)
        nets = self._collect()
        dev = nets[0][0].device
        self.device = dev
        self._nets = nets
        self.params = nets[0] + nets[1]
        self._validate(self.params)
        self.grad = torch.zeros(_abi.FS_PPO_ACTOR_PARAMS + _abi.FS_PPO_CRITIC_PARAMS, dtype=torch.float32, device=dev)
        off = 0
        for p in self.params:
            p.grad = self.grad[off:off + p.numel()].view_as(p)
            off += p.numel()
        assert off == self.grad.numel()
        self.loss = torch.zeros(3, dtype=torch.float32, device=dev)
        self.workspace = torch.empty(lib().fs_ppo_workspace_bytes(), dtype=torch.uint8, device=dev)
        self._bind()

    def _collect(self):
        """The parameters as the modules hold them now: [weight, bias] x 3 per network (a module
        whose weight was replaced -- load_state_dict(assign=True), m.weight = nn.Parameter(...) --
        yields the new tensor)."""
        torch = _torch()
        nets = []
        for net, out in zip(self._modules, (N_ACTIONS, 1)):
            lin = [m for m in net if isinstance(m, torch.nn.Linear)]
            acts = [m for m in net if not isinstance(m, torch.nn.Linear)]
            shapes = [tuple(m.weight.shape) for m in lin]
            if shapes != [(64, N_FEATURES), (64, 64), (out, 64)] or not all(isinstance(m, torch.nn.Tanh) for m in acts):
                raise ValueError("the fused learner takes 8-64-64-%d tanh MLPs; got %s" % (out, shapes))
            if any(m.bias is None for m in lin):
                raise ValueError("the fused learner needs every Linear to have a bias")
            nets.append([t for m in lin for t in (m.weight, m.bias)])
        return nets

    def _validate(self, params):
        torch = _torch()
        for t in params:
            if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
                raise ValueError("the fused learner needs contiguous fp32 device parameters")
            if t.device != self.device:
                raise ValueError("parameter on %s, but the fused learner was built on %s" % (t.device, self.device))

    def _bind(self):
        """The kernels' view of the parameters: raw device pointers of every weight and bias."""
        self._mlps = [_abi.fs_mlp(*[t.data_ptr() for t in params]) for params in self._nets]
        self._ptrs = [p.data_ptr() for p in self.params]

    def _check_bindings(self):
        """Before a launch: the parameters are re-collected from the modules (a module whose weight
        or bias was replaced by a new tensor is seen), each must still be a contiguous fp32 tensor
        on this learner's device, every .grad must still be its view of the flat buffer the kernel
        writes (an optimizer's zero_grad(set_to_none=True) drops it; it is re-attached -- the
        kernel overwrites the whole buffer), and the kernel's pointers are re-read when any
        parameter moved (param.data = ..., a new Parameter)."""
        nets = self._collect()
        params = nets[0] + nets[1]
        moved = [p.data_ptr() for p in params] != self._ptrs or any(a is not b for a, b in zip(params, self.params))
        if moved:
            self._validate(params)
            self._nets, self.params = nets, params
        off = 0
        base = self.grad.data_ptr()
        for p in self.params:
            if p.grad is None or p.grad.data_ptr() != base + 4 * off or p.grad.shape != p.shape:
                p.grad = self.grad[off:off + p.numel()].view_as(p)
            off += p.numel()
        if moved:
            self._bind()

    def evaluate(self, x, actions=None, n_logp=0, precision=None, values=True):
        """fs_ppo_eval: (critic(x) [n], log_softmax(actor(x[:n_logp]))[actions] [n_logp] or None),
        without gradient; x: device [n, 8] fp32, actions: device uint8 [n_logp].  `precision`:
        "fp32" or "split_bf16" for this call (default: the learner's own); values=False: the
        log-probs only (the critic is not run, the first result is None)."""
        torch = _torch()
        if precision is not None and precision not in self.PRECISIONS:
            raise ValueError("precision must be one of %s" % sorted(self.PRECISIONS))
        prec = self._prec if precision is None else self.PRECISIONS[precision]
        if x.dtype != torch.float32 or x.dim() != 2 or x.shape[1] != N_FEATURES or not x.is_contiguous():
            raise ValueError("x must be a contiguous [n, 8] float32 tensor")
        n = x.shape[0]
        want_values = values
        values = torch.empty(n, dtype=torch.float32, device=x.device) if want_values else None
        logp = None
        if n_logp:
            if actions is None or actions.dtype != torch.uint8 or actions.numel() < n_logp or not actions.is_contiguous():
                raise ValueError("actions must be a contiguous uint8 tensor of at least n_logp entries")
            logp = torch.empty(n_logp, dtype=torch.float32, device=x.device)
        self._check_bindings()
        stream = torch.cuda.current_stream(self.device).cuda_stream
        check(lib().fs_ppo_eval_ex(C.c_void_p(x.data_ptr()), n, C.c_void_p(actions.data_ptr() if n_logp else None),
                                   n_logp, C.byref(self._mlps[0]), C.byref(self._mlps[1]),
                                   C.c_void_p(values.data_ptr() if want_values else None),
                                   C.c_void_p(logp.data_ptr() if n_logp else None),
                                   C.c_void_p(self.workspace.data_ptr()), self.workspace.numel(), C.c_void_p(stream),
                                   prec))
        return values, logp

    def __call__(self, rows, clip, vf_coef, ent_coef, runs=None, run_len=1):
        """rows: device [n][12] fp32 (features, action, old log-prob, advantage, return).  With
        `runs` (device int64 [k]) the minibatch is the k runs rows[runs[j] * run_len :
        (runs[j] + 1) * run_len] in that order, read in place (fs_ppo_grad_runs; run_len a power
        of two): the same gradient, bit for bit, as on ``rows.view(-1, run_len, 12)[runs]``."""
        torch = _torch()
        if rows.dtype != torch.float32 or rows.dim() != 2 or rows.shape[1] != 12 or not rows.is_contiguous():
            raise ValueError("rows must be a contiguous [n, 12] float32 tensor")
        self._check_bindings()
        stream = torch.cuda.current_stream(self.device).cuda_stream
        tail = (C.byref(self._mlps[0]), C.byref(self._mlps[1]), clip, vf_coef, ent_coef,
                C.c_void_p(self.grad.data_ptr()), C.c_void_p(self.loss.data_ptr()),
                C.c_void_p(self.workspace.data_ptr()), self.workspace.numel(), C.c_void_p(stream), self._prec)
        if runs is None:
            check(lib().fs_ppo_grad_ex(C.c_void_p(rows.data_ptr()), rows.shape[0], *tail))
            return self.loss
        shift = int(run_len).bit_length() - 1
        if run_len < 1 or (1 << shift) != run_len:
            raise ValueError("run_len must be a power of two")
        if runs.dtype != torch.int64 or runs.dim() != 1 or not runs.is_contiguous() or runs.device != rows.device:
            raise ValueError("runs must be a contiguous int64 vector on the rows' device")
        check(lib().fs_ppo_grad_runs(C.c_void_p(rows.data_ptr()), rows.shape[0], C.c_void_p(runs.data_ptr()),
                                     runs.numel(), shift, *tail))
        return self.loss


def gae(rewards, values, dones, gamma, lam):
    """Generalised advantage estimation over [T][N]: values has T + 1 rows (the last one
    bootstraps); dones[t] = 1 cuts the recursion after tick t.  Returns (advantages, returns)."""
    torch = _torch()
    T = rewards.shape[0]
    keep = 1.0 - dones
    delta = rewards + gamma * values[1:] * keep - values[:-1]  # every tick's TD error at once
    coef = (gamma * lam) * keep
    adv = torch.empty_like(rewards)
    adv[T - 1] = delta[T - 1]
    for t in range(T - 2, -1, -1):  # the backward recursion: one fused multiply-add per tick
        torch.addcmul(delta[t], coef[t], adv[t + 1], out=adv[t])
    return adv, adv + values[:-1]


def gae_device(rewards, dones, values, gamma, lam):
    """gae() in one launch (fs_ppo_gae): rewards [T][N] f64 and dones [T][N] u8 as the trajectory
    holds them, values [T + 1][N] f32; the TD errors in gae()'s op order, the recursion as a fused
    multiply-add (addcmul's), so the two agree to fp32 rounding of that step."""
    torch = _torch()
    T, N = rewards.shape
    if (rewards.dtype != torch.float64 or dones.dtype != torch.uint8 or values.dtype != torch.float32
            or tuple(dones.shape) != (T, N) or tuple(values.shape) != (T + 1, N)
            or not all(t.is_contiguous() for t in (rewards, dones, values))):
        raise ValueError("gae_device: contiguous rewards f64 [T][N], dones u8 [T][N], values f32 [T+1][N]")
    adv = torch.empty((T, N), dtype=torch.float32, device=values.device)
    ret = torch.empty_like(adv)
    g = torch.tensor([gamma, gamma * lam], dtype=torch.float32)  # the f32 scalars torch's ops use
    stream = torch.cuda.current_stream(values.device).cuda_stream
    check(lib().fs_ppo_gae(C.c_void_p(rewards.data_ptr()), C.c_void_p(dones.data_ptr()), C.c_void_p(values.data_ptr()),
                           T, N, float(g[0]), float(g[1]), C.c_void_p(adv.data_ptr()), C.c_void_p(ret.data_ptr()),
                           C.c_void_p(stream)))
    return adv, ret


def features_device(tr, out):
    """obs_features of every [T][N] trajectory row in one launch (fs_ppo_features) into out
    [T][N][8] f32, bit-identical to the torch ops (each division by a host scalar is torch's
    x * f32(1 / b), the reciprocal taken in f64)."""
    torch = _torch()
    cols = (tr["guard"], tr["move"], tr["move_frame"], tr["position"])
    n = out.numel() // N_FEATURES
    if (out.dtype != torch.float32 or not out.is_contiguous() or out.shape[-1] != N_FEATURES
            or not all(t.is_contiguous() and t.numel() == 2 * n for t in cols)
            or cols[0].dtype != torch.uint8 or cols[1].dtype != torch.uint8
            or cols[2].dtype != torch.float32 or cols[3].dtype != torch.float32):
        raise ValueError("features_device: contiguous u8 guard / move, f32 move_frame / position [..][2], f32 out [..][8]")
    stream = torch.cuda.current_stream(out.device).cuda_stream
    check(lib().fs_ppo_features(*[C.c_void_p(t.data_ptr()) for t in cols], n, C.c_void_p(out.data_ptr()),
                                C.c_void_p(stream)))
    return out


def pack_rows(x, actions, old, adv, ret, out=None, stats=None):
    """fs_ppo_grad's [M, 12] sample table in one launch (fs_ppo_pack): x [M, 8] f32, actions u8
    [M], old log-probs, advantages and returns f32 [M]; the advantages normalised on the way as
    (adv - mean) / (std + 1e-8) with torch's mean and (unbiased) std -- or with `stats` (a device
    f32 [2]: mean, std), data-parallel PPO's statistics over every rank's advantages."""
    torch = _torch()
    M = x.shape[0]
    if (x.dtype != torch.float32 or tuple(x.shape) != (M, N_FEATURES) or actions.dtype != torch.uint8
            or not all(t.is_contiguous() and t.numel() == M for t in (actions, old, adv, ret))
            or not x.is_contiguous()):
        raise ValueError("pack_rows: contiguous x f32 [M, 8], actions u8 [M], old / adv / ret f32 [M]")
    if stats is None:
        stats = torch.stack([adv.mean(), adv.std()])
    rows = out if out is not None else torch.empty((M, 12), dtype=torch.float32, device=x.device)
    stream = torch.cuda.current_stream(x.device).cuda_stream
    check(lib().fs_ppo_pack(C.c_void_p(x.data_ptr()), C.c_void_p(actions.data_ptr()), C.c_void_p(old.data_ptr()),
                            C.c_void_p(adv.data_ptr()), C.c_void_p(ret.data_ptr()), C.c_void_p(stats.data_ptr()), M,
                            C.c_void_p(rows.data_ptr()), C.c_void_p(stream)))
    return rows


class PPOTrainer:
    """PPO over a FootsiesSim (P2 = whatever the sim was created with).  `horizon` ticks per
    rollout, all arenas in every minibatch round.  `learner_precision` is PPOGrad's: the
    split-bf16 hidden layer by default -- against a float64 autograd reference its gradients are
    within 5e-6 of each tensor's largest entry, as close as torch's own fp32 autograd (up to
    1.1e-5; profiles/r04e_split_error.jsonl) -- or "fp32".

    Data-parallel (`group`: a torch.distributed process group, or "default" for the default one;
    SURVEY.md §8(e)): one trainer per rank, each over its own FootsiesSim (a ShardedSim's handle:
    its arena_base keys the actor's sampling stream, so ranks roll out different arenas), all with
    the same `num_envs`.  The ranks start from rank 0's weights; rollouts, GAE and the sample table
    stay rank-local, the advantages are normalised with the statistics of every rank's advantages
    (parallel.global_mean_std), and each minibatch's gradient -- the mean over this rank's share of
    it -- is averaged over the ranks (parallel.allreduce_mean_, one all_reduce of the flat gradient
    buffer over RCCL) before the Adam step, so every rank applies the same update to the same
    weights: G ranks x N arenas train one policy on G x N arenas' samples per iteration."""

    def __init__(self, sim, actor=None, critic=None, horizon=128, gamma=0.99, lam=0.95, epochs=2, minibatches=4,
                 lr=3e-4, clip=0.2, vf_coef=0.5, ent_coef=0.01, seed=0, old_logp="behaviour", learner="hip",
                 kl_ticks=None, learner_precision="split_bf16", group=None):
        torch = _torch()
        if old_logp not in ("behaviour", "fp32"):
            raise ValueError("old_logp must be 'behaviour' or 'fp32'")
        if learner not in ("hip", "torch"):
            raise ValueError("learner must be 'hip' or 'torch'")
        if int(epochs) < 1 or int(minibatches) < 1 or int(horizon) < 1:
            raise ValueError("PPOTrainer needs epochs >= 1, minibatches >= 1 and horizon >= 1")
        self.learner = learner
        self.old_logp = old_logp
        dev = sim.device
        self.sim = sim
        self.actor = actor if actor is not None else make_actor(device=dev, seed=seed)
        self.critic = critic if critic is not None else make_critic(device=dev, seed=seed + 1)
        self.group, self.world = None, 1
        if group is not None:
            import torch.distributed as dist
            self.group = None if group == "default" else group
            self.world = dist.get_world_size(self.group)
        if self.world > 1:
            self._join_ranks(sim.num_envs)
        self.rollout = FusedPolicyRollout(sim, self.actor, seed=seed)
        self.horizon, self.gamma, self.lam = horizon, gamma, lam
        # the fp32 log-probs behind kl_behaviour_fp32 / logp_abs_diff: every tick when they are
        # PPO's old log-probs, else a sample of the first `kl_ticks` ticks (all arenas)
        self.kl_ticks = horizon if old_logp == "fp32" else min(horizon, kl_ticks or max(1, horizon // 16))
        self.epochs, self.minibatches, self.clip = epochs, minibatches, clip
        self.vf_coef, self.ent_coef = vf_coef, ent_coef
        # one fused kernel per step on the device instead of ~7 foreach launches
        self.opt = torch.optim.Adam(list(self.actor.parameters()) + list(self.critic.parameters()), lr=lr,
                                    fused=dev.type == "cuda")
        self._grad = PPOGrad(self.actor, self.critic, precision=learner_precision) if learner == "hip" else None
        self.traj = sim.alloc_trajectory(horizon)
        n = sim.num_envs
        self.actions = torch.empty((horizon, n), dtype=torch.uint8, device=dev)
        self.logp = torch.empty((horizon, n), dtype=torch.float32, device=dev)
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(seed)
        self.stats = {}
        # the observation before the next rollout's first tick: the sim's outputs now, then
        # the last trajectory row (trajectory launches leave the regular outputs untouched)
        self._next_first = None

    def _join_ranks(self, n):
        """Data-parallel start: the same arena count on every rank (each minibatch step is one
        collective per rank, so the ranks must take the same number of them) and rank 0's weights."""
        import torch.distributed as dist
        from .parallel import _on_backend
        torch = _torch()
        counts = [None] * self.world
        dist.all_gather_object(counts, int(n), group=self.group)
        if len(set(counts)) != 1:
            raise ValueError("data-parallel PPO needs the same num_envs on every rank, got %s" % counts)
        src = dist.get_global_rank(self.group, 0) if self.group is not None else 0
        with torch.no_grad():
            for p in list(self.actor.parameters()) + list(self.critic.parameters()):
                b = _on_backend(p.data, self.group)
                dist.broadcast(b, src, group=self.group)
                if b is not p.data:
                    p.data.copy_(b)

    def collect(self):
        """One fused rollout; returns (features [T+1][N][8] f32, actions u8, rewards f64, dones u8)
        as [T][N] device tensors (the trajectory's own buffers)."""
        torch = _torch()
        first = self._next_first if self._next_first is not None else obs_features(self.sim.outputs())
        self.rollout.rollout(self.horizon, self.actions, self.logp, trajectory=self.traj)
        cur = torch.cuda.current_stream(self.sim.device)
        if cur != self.sim.stream:  # the trajectory was written on the handle's stream
            cur.wait_stream(self.sim.stream)
        tr = self.traj
        T, N = self.horizon, self.sim.num_envs
        feats = torch.empty((T + 1, N, N_FEATURES), dtype=torch.float32, device=first.device)
        feats[0] = first
        if self._grad is not None:
            features_device(tr, feats[1:])  # obs_features of every tick, one launch
        else:
            f = feats[1:]  # each pair written into its columns
            torch.div(tr["guard"], 3.0, out=f[..., 0:2])
            torch.div(tr["move"], 16.0, out=f[..., 2:4])
            torch.div(tr["move_frame"], 55.0, out=f[..., 4:6])
            torch.div(tr["position"], 4.6, out=f[..., 6:8])
        self._next_first = feats[T]
        return feats, self.actions, tr["reward"], tr["terminated"]

    def prepare(self, feats, actions, rewards, dones):
        """The sample table of one rollout: (rows [T*N][12] -- features, action, old log-prob,
        advantage, return --, gap = behaviour log-prob - fp32 log-prob over the KL samples)."""
        torch = _torch()
        T, N = actions.shape
        M = T * N
        nk = self.kl_ticks * N  # samples with an fp32 log-prob (all of them in "fp32" mode)
        with torch.no_grad():
            x = feats[:T].reshape(M, N_FEATURES)
            a = actions.reshape(M)
            behav = self.logp.reshape(M)  # what the kernel sampled with (bf16 actor)
            if self._grad is not None:  # the forward passes, GAE and the sample table
                # old32 -- the fp32 reference the KL diagnostic and old_logp="fp32" are defined
                # against -- always at fp32 FMAs, whatever the learner's precision; the critic values
                # (GAE's baseline) always at the learner's own precision, whatever old_logp is (one
                # call serves both when the learner is fp32 and every sample needs its log-prob)
                if nk == M and self._grad.precision == "fp32":
                    v, old32 = self._grad.evaluate(feats.view(-1, N_FEATURES), a, nk)
                else:
                    v, _ = self._grad.evaluate(feats.view(-1, N_FEATURES))
                    _, old32 = self._grad.evaluate(x[:nk].contiguous(), a, nk, precision="fp32", values=False)
                values = v.view(T + 1, N)
                adv, ret = gae_device(rewards, dones, values, self.gamma, self.lam)
                old = behav if self.old_logp == "behaviour" else old32
                rows = pack_rows(x, a, old, adv.view(M), ret.view(M), stats=self._adv_stats(adv))
            else:
                values = self.critic(feats).squeeze(-1)  # [T+1][N]
                old32 = torch.log_softmax(self.actor(x[:nk]), dim=1).gather(1, a[:nk, None].long())[:, 0]
                adv, ret = gae(rewards.float(), values, dones.float(), self.gamma, self.lam)
                old = behav if self.old_logp == "behaviour" else old32
                adv = adv.reshape(M)
                st = self._adv_stats(adv)
                if st is None:
                    adv = (adv - adv.mean()) / (adv.std() + 1e-8)
                else:
                    adv = (adv - st[0]) / (st[1] + 1e-8)
                rows = torch.cat([x, a[:, None].float(), old[:, None], adv[:, None], ret.reshape(M, 1)], dim=1)  # [M, 12]
            gap = behav[:nk] - old32
        return rows, gap

    def _adv_stats(self, adv):
        """The advantage normalisation's (mean, std) over every rank (data-parallel), else None
        (this rank's own, as pack_rows / the torch learner compute them)."""
        if self.world == 1:
            return None
        from .parallel import global_mean_std
        return global_mean_std(adv, self.group)

    def _average_grads(self):
        """Data-parallel: this minibatch's gradient averaged over the ranks before the step."""
        if self.world == 1:
            return
        from .parallel import allreduce_mean_
        if self._grad is not None:
            allreduce_mean_(self._grad.grad, self.group)  # the flat buffer the .grad views share
            return
        torch = _torch()
        ps = [p for p in list(self.actor.parameters()) + list(self.critic.parameters()) if p.grad is not None]
        flat = torch.cat([p.grad.reshape(-1) for p in ps])
        allreduce_mean_(flat, self.group)
        off = 0
        for p in ps:
            p.grad.copy_(flat[off:off + p.numel()].view_as(p.grad))
            off += p.numel()

    def update(self, feats, actions, rewards, dones):
        torch = _torch()
        T, N = actions.shape
        M = T * N
        rows, gap = self.prepare(feats, actions, rewards, dones)
        # Minibatches: a random permutation of runs of _SHUFFLE_CHUNK consecutive samples (one tick,
        # that many consecutive arenas) when they tile the batch, so each minibatch is gathered as
        # whole runs (row copies) instead of 2 M scattered rows; per-sample otherwise.
        C = _SHUFFLE_CHUNK if M % (_SHUFFLE_CHUNK * self.minibatches) == 0 else 1
        runs = rows.view(M // C, C, rows.shape[1])
        nb = (M // C + self.minibatches - 1) // self.minibatches
        for _ in range(self.epochs):
            perm = torch.randperm(M // C, device=rows.device, generator=self.gen)
            for i in range(0, M // C, nb):
                if self._grad is not None:  # fused forward + backward straight into .grad, the runs read in place
                    lm = self._grad(rows, self.clip, self.vf_coef, self.ent_coef, runs=perm[i:i + nb], run_len=C)
                    self._average_grads()
                    self.opt.step()
                    continue
                b = runs[perm[i:i + nb]].view(-1, rows.shape[1])
                xb, ab = b[:, :N_FEATURES], b[:, N_FEATURES].long()
                oldb, advb, retb = b[:, N_FEATURES + 1], b[:, N_FEATURES + 2], b[:, N_FEATURES + 3]
                logits = mlp(self.actor, xb)
                lp_all = torch.log_softmax(logits, dim=1)
                lp = lp_all.gather(1, ab[:, None])[:, 0]
                ratio = torch.exp(lp - oldb)
                s1, s2 = ratio * advb, torch.clamp(ratio, 1 - self.clip, 1 + self.clip) * advb
                pg = -torch.min(s1, s2).mean()
                vf = (mlp(self.critic, xb).squeeze(-1) - retb).pow(2).mean()
                ent = -(lp_all.exp() * lp_all).sum(1).mean()
                loss = pg + self.vf_coef * vf - self.ent_coef * ent
                self.opt.zero_grad(set_to_none=True)
                loss.backward()
                self._average_grads()
                self.opt.step()
        self.rollout.refresh(self.actor)
        if self._grad is not None:
            pg, vf, ent = lm[0].clone(), lm[1].clone(), lm[2].clone()
            loss = pg + self.vf_coef * vf - self.ent_coef * ent
        if self.world > 1:  # the last minibatch's losses, averaged like its gradient
            from .parallel import allreduce_mean_
            torch = _torch()
            red = allreduce_mean_(torch.stack([loss.detach(), pg.detach(), vf.detach(), ent.detach()]), self.group)
            loss, pg, vf, ent = red[0], red[1], red[2], red[3]
        self.stats = {"loss": loss.detach(), "policy_loss": pg.detach(), "value_loss": vf.detach(),
                      "entropy": ent.detach(), "mean_reward": rewards.mean(), "kl_behaviour_fp32": gap.mean(),
                      "logp_abs_diff": gap.abs().mean()}

    def iterate(self):
        self.update(*self.collect())

    def train(self, iterations, sync=True):
        """Run `iterations` PPO iterations; returns env-steps/s of the whole loop (rollout +
        learning), timed around device synchronisation."""
        torch = _torch()
        torch.cuda.synchronize(self.sim.device)
        t0 = time.perf_counter()
        for _ in range(iterations):
            self.iterate()
        if sync:
            torch.cuda.synchronize(self.sim.device)
        return iterations * self.horizon * self.sim.num_envs / (time.perf_counter() - t0)


__all__ = ["PPOTrainer", "PPOGrad", "make_critic", "gae", "gae_device", "pack_rows", "features_device", "N_ACTIONS"]
