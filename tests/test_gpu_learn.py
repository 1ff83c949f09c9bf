"""fs_ppo_grad (csrc/fs_learn.hip), the C5 learner's fused forward + backward, against torch
autograd on the same loss (ppo.py's learner="torch" path, written out here): fp32 gradients of
both networks and the three loss means, on ragged sample counts (a partial last 64-sample
tile), with ratios inside and outside the clip range (none within 1e-3 of a clip edge, see
_rows) and a zero-advantage tie.  Both learner precisions: "fp32" (fp32 FMAs) and "split_bf16"
(PPOTrainer's default: the hidden layer on bf16 MFMAs, each fp32 operand split hi + lo).

Tolerance: the kernel and hipBLASLt sum in different orders in fp32, so each gradient tensor
must agree to rtol 1e-4 with atol 1e-6 x that tensor's largest magnitude (measured differences
are ~1e-6 relative).  split_bf16 drops the lo*lo term of every hidden-layer product (2^-16
relative of it) before fp32 accumulation: the same rtol, atol 1e-5 x the largest magnitude.
Not a bit-exact path: this is the learner beside the simulator."""
import pytest

pytestmark = pytest.mark.gpu

RTOL = 1e-4
ATOL_FRAC = {"fp32": 1e-6, "split_bf16": 1e-5}
PRECISIONS = ("fp32", "split_bf16")


def _nets(seed):
    import torch
    from footsies_gym_amd.ppo import make_critic
    from footsies_gym_amd.rollout import make_actor
    dev = torch.device("cuda", 0)
    return make_actor(device=dev, seed=seed), make_critic(device=dev, seed=seed + 1)


def _rows(actor, n, seed, margin=1e-3, clip=0.2):
    """[n, 12] rows whose old log-probs put ratios below, inside and above the clip range, none
    within `margin` of a clip edge: there the clipped loss's gradient jumps (the sample's policy
    term switches on or off), so any rounding difference in the forward pass can flip a sample
    and move the minibatch gradient by ~1/sqrt(n) relative -- a property of the loss, not of
    the kernel (measured with the float64 reference: tools/split_error.py)."""
    import torch
    g = torch.Generator(device="cuda").manual_seed(seed)
    dev = torch.device("cuda", 0)
    x = torch.rand((n, 8), generator=g, device=dev) * 2 - 0.5
    a = torch.randint(0, 8, (n,), generator=g, device=dev)
    with torch.no_grad():
        lp = torch.log_softmax(actor(x), dim=1).gather(1, a[:, None])[:, 0]
    old = lp + torch.randn(n, generator=g, device=dev) * 0.3
    for edge in (1 - clip, 1 + clip):  # ratio = exp(lp - old): move old so it sits 2 margins away
        near = (torch.exp(lp - old) - edge).abs() < margin
        old = torch.where(near, lp - torch.log(torch.full_like(old, edge + 2 * margin)), old)
    adv = torch.randn(n, generator=g, device=dev)
    adv[::17] = 0.0  # s1 == s2 == 0: torch.min's tie
    ret = torch.randn(n, generator=g, device=dev)
    return torch.cat([x, a[:, None].float(), old[:, None], adv[:, None], ret[:, None]], dim=1).contiguous()


def _torch_reference(actor, critic, rows, clip, vf_coef, ent_coef):
    """ppo.py's update loss on one minibatch, through autograd (the learner="torch" path)."""
    import torch
    xb, ab = rows[:, :8], rows[:, 8].long()
    oldb, advb, retb = rows[:, 9], rows[:, 10], rows[:, 11]
    params = list(actor.parameters()) + list(critic.parameters())
    for p in params:
        p.grad = None
    lp_all = torch.log_softmax(actor(xb), dim=1)
    lp = lp_all.gather(1, ab[:, None])[:, 0]
    ratio = torch.exp(lp - oldb)
    pg = -torch.min(ratio * advb, torch.clamp(ratio, 1 - clip, 1 + clip) * advb).mean()
    vf = (critic(xb).squeeze(-1) - retb).pow(2).mean()
    ent = -(lp_all.exp() * lp_all).sum(1).mean()
    (pg + vf_coef * vf - ent_coef * ent).backward()
    grads = [p.grad.detach().clone() for p in params]
    for p in params:
        p.grad = None
    return grads, torch.stack([pg, vf, ent]).detach()


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("n", [1, 63, 64, 5000, 70001])
def test_ppo_grad_matches_autograd(n, precision):
    import torch
    from footsies_gym_amd.ppo import PPOGrad
    actor, critic = _nets(seed=n % 7)
    rows = _rows(actor, n, seed=n)
    clip, vf_coef, ent_coef = 0.2, 0.5, 0.01
    ref, ref_loss = _torch_reference(actor, critic, rows, clip, vf_coef, ent_coef)
    pg = PPOGrad(actor, critic, precision=precision)
    loss = pg(rows, clip, vf_coef, ent_coef).clone()
    got = [p.grad.detach().clone() for p in pg.params]
    torch.cuda.synchronize()
    r = torch.exp(torch.log_softmax(actor(rows[:, :8]), 1).gather(1, rows[:, 8].long()[:, None])[:, 0] - rows[:, 9])
    if n >= 5000:  # the rows exercise both clip edges
        assert bool((r < 1 - clip).any()) and bool((r > 1 + clip).any()) and bool(((r > 0.8) & (r < 1.2)).any())
    names = ["actor.w1", "actor.b1", "actor.w2", "actor.b2", "actor.w3", "actor.b3",
             "critic.w1", "critic.b1", "critic.w2", "critic.b2", "critic.w3", "critic.b3"]
    for name, g, e in zip(names, got, ref):
        assert g.shape == e.shape, name
        scale = float(e.abs().max())
        torch.testing.assert_close(g, e, rtol=RTOL, atol=ATOL_FRAC[precision] * max(scale, 1e-12),
                                   msg=lambda m, name=name: name + ": " + m)
    torch.testing.assert_close(loss, ref_loss, rtol=RTOL, atol=1e-6)


@pytest.mark.parametrize("precision", PRECISIONS)
def test_ppo_grad_is_deterministic_and_rejects_bad_input(precision):
    import torch
    from footsies_gym_amd._lib import FootsiesError
    from footsies_gym_amd.ppo import PPOGrad
    from footsies_gym_amd.rollout import make_actor
    actor, critic = _nets(seed=2)
    rows = _rows(actor, 200_000, seed=9)
    pg = PPOGrad(actor, critic, precision=precision)
    pg(rows, 0.2, 0.5, 0.01)
    first = pg.grad.clone()
    pg(rows, 0.2, 0.5, 0.01)
    assert torch.equal(first, pg.grad)  # fixed summation order: identical on every call
    with pytest.raises(ValueError):
        pg(rows[:, :11].contiguous(), 0.2, 0.5, 0.01)
    with pytest.raises(FootsiesError):
        pg(rows[:0], 0.2, 0.5, 0.01)
    with pytest.raises(ValueError):
        PPOGrad(make_actor(hidden=32, device=torch.device("cuda", 0)), critic)
    with pytest.raises(ValueError):
        PPOGrad(actor, critic, precision="bf16")


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("run_len,n_runs", [(2048, 37), (1, 5001), (16, 333)])
def test_ppo_grad_over_runs_equals_gathered_rows(precision, run_len, n_runs):
    """fs_ppo_grad_runs (PPOTrainer.update's minibatches: shuffled runs of consecutive samples read
    in place) against fs_ppo_grad_ex on the same runs gathered into a table first: the gradient and
    the loss means bit for bit -- run lengths of whole tiles (2048, PPOTrainer's), single samples
    and runs shorter than a tile (16), with a partial last tile; then out-of-table run entries
    read as padding rows and the host-side argument checks."""
    import torch
    from footsies_gym_amd._lib import FootsiesError
    from footsies_gym_amd.ppo import PPOGrad
    actor, critic = _nets(seed=3)
    total = 64 * 2048
    rows = _rows(actor, total, seed=11)
    g = torch.Generator(device="cuda").manual_seed(run_len + n_runs)
    runs = torch.randperm(total // run_len, generator=g, device="cuda")[:n_runs].contiguous()
    pg = PPOGrad(actor, critic, precision=precision)
    gathered = rows.view(-1, run_len, 12)[runs].reshape(-1, 12).contiguous()
    loss_g = pg(gathered, 0.2, 0.5, 0.01).clone()
    grad_g = pg.grad.clone()
    loss_r = pg(rows, 0.2, 0.5, 0.01, runs=runs, run_len=run_len).clone()
    assert torch.equal(grad_g, pg.grad) and torch.equal(loss_g, loss_r)
    # a run entry past the table: nothing read, nothing added (the padding rows' zero gradient) --
    # whatever the entry: just past the table, negative, or so large that shifting it by the run
    # length wraps back into the table (1 << 62 at run_len 2048 shifted to row 0)
    outs = []
    for v in (total // run_len + 5, -1, 1 << 62, (1 << 63) - 1):
        bad = runs.clone()
        bad[-1] = v
        loss_b = pg(rows, 0.2, 0.5, 0.01, runs=bad, run_len=run_len).clone()
        assert bool(torch.isfinite(pg.grad).all())
        outs.append((loss_b, pg.grad.clone()))
    for loss_b, grad_b in outs[1:]:
        assert torch.equal(loss_b, outs[0][0]) and torch.equal(grad_b, outs[0][1])
    if n_runs > 1:  # the padding run differs from the real run it replaced
        assert not torch.equal(outs[0][1], grad_g)
    with pytest.raises(ValueError):
        pg(rows, 0.2, 0.5, 0.01, runs=runs, run_len=3)
    with pytest.raises(ValueError):
        pg(rows, 0.2, 0.5, 0.01, runs=runs.int(), run_len=run_len)
    with pytest.raises(FootsiesError):
        pg(rows, 0.2, 0.5, 0.01, runs=runs[:0], run_len=run_len)


def test_ppo_trainer_hip_step_equals_torch_step():
    """One minibatch update through PPOTrainer's two learners from the same weights and rows:
    the parameters after Adam agree (Adam's first step moves each weight by ~lr * sign(grad), so
    a sign flip of a near-zero gradient is the only way they could differ by more than
    rounding; it is bounded by 2 lr and counted)."""
    import torch
    from footsies_gym_amd.ppo import PPOGrad
    actor, critic = _nets(seed=5)
    rows = _rows(actor, 32768, seed=5)
    lr = 1e-3
    res = []
    for learner in ("hip", "torch"):
        a, c = _nets(seed=5)
        opt = torch.optim.Adam(list(a.parameters()) + list(c.parameters()), lr=lr)
        if learner == "hip":
            PPOGrad(a, c)(rows, 0.2, 0.5, 0.01)
        else:
            grads, _ = _torch_reference(a, c, rows, 0.2, 0.5, 0.01)
            for p, g in zip(list(a.parameters()) + list(c.parameters()), grads):
                p.grad = g
        opt.step()
        res.append([p.detach().clone() for p in list(a.parameters()) + list(c.parameters())])
    flips = 0
    for h, t in zip(*res):
        d = (h - t).abs()
        assert float(d.max()) <= 2 * lr * 1.001
        flips += int((d > 1e-6).sum())
    total = sum(p.numel() for p in res[0])
    assert flips <= total // 1000, (flips, total)


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("n,n_logp", [(1, 1), (100, 37), (70001, 70001), (131072 + 65536, 131072)])
def test_ppo_eval_matches_torch_forward(n, n_logp, precision):
    """fs_ppo_eval: critic values of every row and the actor's log-probability of the taken action
    for the first n_logp rows, against the torch modules' forward pass (fp32, same tolerance)."""
    import torch
    from footsies_gym_amd.ppo import PPOGrad
    actor, critic = _nets(seed=3)
    g = torch.Generator(device="cuda").manual_seed(n)
    x = (torch.rand((n, 8), generator=g, device="cuda") * 2 - 0.5).contiguous()
    a = torch.randint(0, 8, (n_logp,), generator=g, device="cuda").to(torch.uint8)
    v, lp = PPOGrad(actor, critic, precision=precision).evaluate(x, a, n_logp)
    with torch.no_grad():
        v_ref = critic(x).squeeze(-1)
        lp_ref = torch.log_softmax(actor(x[:n_logp]), 1).gather(1, a.long()[:, None])[:, 0]
    torch.testing.assert_close(v, v_ref, rtol=RTOL, atol=1e-5)
    torch.testing.assert_close(lp, lp_ref, rtol=RTOL, atol=1e-5)
    v2, lp2 = PPOGrad(actor, critic, precision=precision).evaluate(x)
    assert lp2 is None and torch.equal(v2, v)


@pytest.mark.parametrize("T,N", [(1, 5), (17, 333), (128, 4096)])
def test_ppo_gae_and_pack_match_torch(T, N):
    """fs_ppo_gae against ppo.gae (the TD errors op for op; the recursion's fused multiply-add
    against addcmul: rtol 1e-5, atol 1e-5 x the largest advantage), and fs_ppo_pack against the
    torch.cat sample table with torch's normalisation: bit-exact on the same advantages."""
    import torch
    from footsies_gym_amd.ppo import gae, gae_device, pack_rows
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cuda").manual_seed(T * 1000 + N)
    rew = torch.randn((T, N), generator=g, device=dev, dtype=torch.float64) * 0.3
    rew[torch.rand((T, N), generator=g, device=dev) < 0.7] = 0.0
    done = (torch.rand((T, N), generator=g, device=dev) < 0.05).to(torch.uint8)
    val = torch.randn((T + 1, N), generator=g, device=dev)
    adv, ret = gae_device(rew, done, val, 0.99, 0.95)
    want_adv, want_ret = gae(rew.float(), val, done.float(), 0.99, 0.95)
    tol = 1e-5 * float(want_adv.abs().max())
    assert torch.allclose(adv, want_adv, rtol=1e-5, atol=tol)
    assert torch.allclose(ret, want_ret, rtol=1e-5, atol=tol)
    if T == 1:  # no recursion: every step is one rounding per op, as in gae()
        assert torch.equal(adv, want_adv) and torch.equal(ret, want_ret)
    M = T * N
    x = torch.rand((M, 8), generator=g, device=dev)
    a = torch.randint(0, 8, (M,), generator=g, device=dev, dtype=torch.uint8)
    old = torch.randn(M, generator=g, device=dev)
    if M < 2:
        return  # (torch's std of one sample is nan; the trainer's batches are large)
    rows = pack_rows(x, a, old, adv.view(M), ret.view(M))
    an = adv.view(M)
    an = (an - an.mean()) / (an.std() + 1e-8)
    want = torch.cat([x, a[:, None].float(), old[:, None], an[:, None], ret.view(M, 1)], dim=1)
    assert torch.equal(rows, want)
    with pytest.raises(ValueError):
        pack_rows(x, a.long(), old, adv.view(M), ret.view(M))
    with pytest.raises(ValueError):
        gae_device(rew.float(), done, val, 0.99, 0.95)


def test_ppo_features_match_obs_features():
    """fs_ppo_features against rollout.obs_features (torch's divisions by host scalars) on every
    trajectory row of a short policy rollout: bit-exact."""
    import torch
    from footsies_gym_amd.ppo import features_device
    from footsies_gym_amd.rollout import FusedPolicyRollout, make_actor, obs_features
    from footsies_gym_amd.simulator import FootsiesSim
    sim = FootsiesSim(3001, p2_mode="bot", seed=11)
    T = 40
    tr = sim.alloc_trajectory(T)
    FusedPolicyRollout(sim, make_actor(device=sim.device, seed=4), seed=2).rollout(T, trajectory=tr)
    out = torch.empty((T, sim.num_envs, 8), dtype=torch.float32, device=sim.device)
    features_device(tr, out)
    for t in (0, 7, T - 1):
        assert torch.equal(out[t], obs_features({k: tr[k][t] for k in ("guard", "move", "move_frame", "position")}))
    with pytest.raises(ValueError):
        features_device(tr, out[:, :, :4])


def test_ppo_grad_follows_replaced_parameters():
    """PPOGrad re-collects the parameters from the modules before every launch (advisor r03): a
    weight replaced by a new Parameter (m.weight = nn.Parameter(...), as load_state_dict(assign=
    True) does) is the one the kernel reads and whose .grad it fills, so the gradient equals the
    fresh learner's on the same weights; a parameter moved off the learner's device is refused."""
    import torch
    from footsies_gym_amd.ppo import PPOGrad
    actor, critic = _nets(seed=3)
    rows = _rows(actor, 4096, seed=3)
    pg = PPOGrad(actor, critic)
    pg(rows, 0.2, 0.5, 0.01)
    lin = [m for m in actor if isinstance(m, torch.nn.Linear)]
    lin[1].weight = torch.nn.Parameter(lin[1].weight.detach() * 0.5 + 0.01)
    loss = pg(rows, 0.2, 0.5, 0.01).clone()
    got = [p.grad.detach().clone() for p in pg.params]
    assert pg.params[2] is lin[1].weight and lin[1].weight.grad is not None
    fresh = PPOGrad(actor, critic)
    ref_loss = fresh(rows, 0.2, 0.5, 0.01).clone()
    torch.cuda.synchronize()
    assert torch.equal(loss, ref_loss)
    for g, e in zip(got, [p.grad for p in fresh.params]):
        assert torch.equal(g, e)
    lin[0].bias = torch.nn.Parameter(lin[0].bias.detach().cpu())
    with pytest.raises(ValueError):
        pg(rows, 0.2, 0.5, 0.01)


def test_split_bf16_eval_agrees_with_fp32_eval():
    """The two precisions' forward passes on the same rows: values and log-probs within rtol 1e-4,
    atol 5e-5 of each other (each hidden-layer product is off by up to ~3 x 2^-17 relative before
    the sums; measured: 3.8e-5 absolute on log-probs near -2), and not identical (the MFMA path ran)."""
    import torch
    from footsies_gym_amd.ppo import PPOGrad
    actor, critic = _nets(seed=6)
    g = torch.Generator(device="cuda").manual_seed(6)
    n = 20000
    x = (torch.rand((n, 8), generator=g, device="cuda") * 2 - 0.5).contiguous()
    a = torch.randint(0, 8, (n,), generator=g, device="cuda").to(torch.uint8)
    v32, lp32 = PPOGrad(actor, critic).evaluate(x, a, n)
    vs, lps = PPOGrad(actor, critic, precision="split_bf16").evaluate(x, a, n)
    torch.testing.assert_close(vs, v32, rtol=1e-4, atol=5e-5)
    torch.testing.assert_close(lps, lp32, rtol=1e-4, atol=5e-5)
    assert not torch.equal(vs, v32) or not torch.equal(lps, lp32)


def test_eval_precision_override_is_the_fp32_path():
    """PPOTrainer's critic values and fp32 old log-probs (the KL diagnostic's reference) come from
    evaluate(precision="fp32") whatever the learner's precision: a split-bf16 learner
    asked for fp32 gives the fp32 learner's values and log-probs bit for bit."""
    import torch
    from footsies_gym_amd.ppo import PPOGrad
    actor, critic = _nets(seed=7)
    g = torch.Generator(device="cuda").manual_seed(7)
    n = 5000
    x = (torch.rand((n, 8), generator=g, device="cuda") * 2 - 0.5).contiguous()
    a = torch.randint(0, 8, (n,), generator=g, device="cuda").to(torch.uint8)
    v32, lp32 = PPOGrad(actor, critic).evaluate(x, a, n)
    split = PPOGrad(actor, critic, precision="split_bf16")
    v, lp = split.evaluate(x, a, n, precision="fp32")
    assert torch.equal(v, v32) and torch.equal(lp, lp32)
    with pytest.raises(ValueError):
        split.evaluate(x, a, n, precision="bf16")


def test_eval_log_probs_without_the_critic():
    """evaluate(values=False) -- PPOTrainer.update's fp32 reference log-probs -- runs only the actor
    (fs_ppo_eval with values_out NULL): the same log-probs, bit for bit, as the call with values."""
    import torch
    from footsies_gym_amd.ppo import PPOGrad
    actor, critic = _nets(seed=4)
    g = torch.Generator(device="cuda").manual_seed(4)
    x = torch.rand((5000, 8), generator=g, device="cuda")
    a = torch.randint(0, 8, (5000,), generator=g, device="cuda").to(torch.uint8)
    for precision in PRECISIONS:
        pg = PPOGrad(actor, critic, precision=precision)
        v, lp = pg.evaluate(x, a, 3001)
        none, lp2 = pg.evaluate(x, a, 3001, values=False)
        assert none is None and v.shape == (5000,) and torch.equal(lp, lp2)
