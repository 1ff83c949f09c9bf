"""fs_step_n_policy: the C5 actor inside the fused tick loop (csrc/fs_policy.h).

Three bars.  The simulation stays bit-exact: the actions the kernel sampled, replayed through
the oracle, give the same per-tick trajectory and final state (also at C5's full 65 536
arenas).  The actor matches its host restatement (tests/policy_ref.py): the same action
wherever the uniform is not within rounding distance of a CDF boundary, and log-probabilities
within 0.05 (bf16 inputs, weights and hidden activations; f32 accumulation).  And it matches the
fp32 torch actor that ppo.py trains within the bf16 tolerances stated at _check_fp32 (measured
at 65 536 x 64: KL estimate 1.5e-5 per tick, mean |d logp| 3e-3, max 0.052)."""
import numpy as np
import pytest

from footsies_gym_amd import _abi
from tests import policy_ref
from tests.parity_utils import compare_outputs, compare_states

pytestmark = pytest.mark.gpu

P2_MODES = {"bot": _abi.FS_P2_BOT, "external": _abi.FS_P2_EXTERNAL, "noop": _abi.FS_P2_NOOP}
AUTORESET = {"same_step": _abi.FS_AUTORESET_SAME_STEP, "next_step": _abi.FS_AUTORESET_NEXT_STEP}
MARGIN = 5e-3  # probability distance from a CDF boundary below which a neighbour may be drawn
LOGP_TOL = 0.05


def _check_policy(params, seed, prev, acts, logps, t0, N):
    """prev: outputs before the first tick; acts/logps: [T][N]; returns the next `prev` source."""
    agreed = checked = 0
    for t in range(len(acts)):
        f = policy_ref.features(prev[t])
        lg = policy_ref.logits(params, f)
        u = policy_ref.policy_uniform(seed, np.arange(N), t0 + t)
        act, logp, margin = policy_ref.sample(lg, u)
        ok = margin > MARGIN
        checked += int(ok.sum())
        agreed += int((act[ok] == acts[t][ok]).sum())
        same = act == acts[t]
        err = np.abs(logp[same] - logps[t][same])
        assert err.max() < LOGP_TOL, (t, float(err.max()))
    assert checked > 0.9 * N * len(acts), checked  # 7 boundaries x 2 x MARGIN ~ 7% fall inside
    assert agreed == checked, "%d of %d actions differ away from CDF boundaries" % (checked - agreed, checked)


@pytest.mark.parametrize("p2,autoreset", [("bot", "same_step"), ("external", "next_step"), ("noop", "same_step")])
def test_fused_policy_matches_oracle_and_actor(oracle_lib, p2, autoreset):
    import torch
    from footsies_gym_amd.rollout import FusedPolicyRollout, make_actor
    from footsies_gym_amd.simulator import FootsiesSim
    N, T1, T2, seed = 3001, 60, 40, 0xC0FFEE  # 2N lanes leave the last wave part-filled
    sim = FootsiesSim(N, p2_mode=p2, autoreset_mode=autoreset, seed=21)
    ora = oracle_lib.Oracle(N, p2_mode=P2_MODES[p2], autoreset_mode=AUTORESET[autoreset], base_seed=21)
    ro = FusedPolicyRollout(sim, make_actor(device=torch.device("cuda", 0), seed=9), seed=seed)
    params = [p.cpu().numpy() for p in ro.params]
    prev0 = sim.outputs_numpy()
    t0 = 0
    for T in (T1, T2):
        p2a = sim.hash_actions(T, seed=5 + t0)[0] if p2 == "external" else None
        traj = sim.alloc_trajectory(T)
        acts, logps = ro.rollout(T, p2_actions=p2a, trajectory=traj)
        torch.cuda.synchronize()
        tr = {k: v.cpu().numpy() for k, v in traj.items()}
        A, LP = acts.cpu().numpy(), logps.cpu().numpy()
        h2 = p2a.cpu().numpy() if p2a is not None else None
        for t in range(T):
            exp = ora.step(A[t], None if h2 is None else h2[t])
            compare_outputs(exp, {k: v[t] for k, v in tr.items()}, step=t0 + t, same_step=autoreset == "same_step")
        prev = [prev0] + [{k: v[t] for k, v in tr.items()} for t in range(T - 1)]
        _check_policy(params, seed, prev, A, LP, t0, N)
        prev0 = {k: v[T - 1] for k, v in tr.items()}
        t0 += T
        assert sim.steps_taken == t0
    assert len(np.unique(A)) == 8
    compare_states(ora.state(), sim.get_state())


# The kernel actor against the fp32 torch actor (rollout.make_actor, what ppo.py trains): bf16
# inputs, weights and hidden activations (8 significant bits each, three layers) with f32
# accumulation.  Bars: the draws agree wherever the uniform is farther than FP32_MARGIN from
# every fp32 CDF boundary; |log p_bf16(a) - log p_fp32(a)| stays below FP32_LOGP_MAX for every
# sample and below FP32_LOGP_MEAN on average; the sample KL estimate below FP32_KL.
FP32_LOGP_MAX = 0.1
FP32_LOGP_MEAN = 0.01
FP32_KL = 1e-3
FP32_MARGIN = 0.02


def _check_fp32(actor, prev, acts, logps, seed, t0, N):
    """Kernel samples / log-probs vs the fp32 actor on the same (f32) features; returns the
    per-tick sample estimate of KL(kernel actor || fp32 actor) and the max |d logp|."""
    import torch
    dev = next(actor.parameters()).device
    kls, worst, agreed, checked, mean_abs = [], 0.0, 0, 0, []
    for t in range(len(acts)):
        f = torch.as_tensor(policy_ref.features(prev[t]), device=dev)
        with torch.no_grad():
            lp32 = torch.log_softmax(actor(f), dim=1).double().cpu().numpy()
        cdf = np.cumsum(np.exp(lp32), axis=1)
        u = policy_ref.policy_uniform(seed, np.arange(N), t0 + t).astype(np.float64)
        a32 = np.minimum((u[:, None] >= cdf).sum(axis=1), 7)
        ok = np.abs(cdf[:, :7] - u[:, None]).min(axis=1) > FP32_MARGIN
        checked += int(ok.sum())
        agreed += int((a32[ok] == acts[t][ok]).sum())
        d = logps[t].astype(np.float64) - lp32[np.arange(N), acts[t]]
        worst = max(worst, float(np.abs(d).max()))
        mean_abs.append(float(np.abs(d).mean()))
        kls.append(float(d.mean()))
    assert checked > 0.6 * N * len(acts), checked
    assert agreed == checked, "%d of %d draws differ from the fp32 actor's away from CDF boundaries" % (
        checked - agreed, checked)
    assert worst < FP32_LOGP_MAX, worst
    assert np.mean(mean_abs) < FP32_LOGP_MEAN, np.mean(mean_abs)
    return kls, worst, float(np.mean(mean_abs))


def test_fused_policy_c5_full_size(oracle_lib):
    """Config C5 at its full size: 65 536 arenas vs the bot, 64 policy-driven ticks in one launch.
    The simulation replays bit-exactly through the oracle (every tick's outputs, the final
    state), the actor matches its bf16 restatement, and the fp32 torch actor within the bf16
    tolerance above; the per-tick KL estimate is reported."""
    import torch
    from footsies_gym_amd.rollout import FusedPolicyRollout, make_actor
    from footsies_gym_amd.simulator import FootsiesSim
    N, T, seed = 65536, 64, 0x5EED5
    sim = FootsiesSim(N, p2_mode="bot", seed=33)
    ora = oracle_lib.Oracle(N, p2_mode=_abi.FS_P2_BOT, base_seed=33)
    actor = make_actor(device=torch.device("cuda", 0), seed=4)
    ro = FusedPolicyRollout(sim, actor, seed=seed)
    prev0 = sim.outputs_numpy()
    traj = sim.alloc_trajectory(T)
    acts, logps = ro.rollout(T, trajectory=traj)
    torch.cuda.synchronize()
    tr = {k: v.cpu().numpy() for k, v in traj.items()}
    A, LP = acts.cpu().numpy(), logps.cpu().numpy()
    for t in range(T):
        compare_outputs(ora.step(A[t]), {k: v[t] for k, v in tr.items()}, step=t)
    compare_states(ora.state(), sim.get_state())
    prev = [prev0] + [{k: v[t] for k, v in tr.items()} for t in range(T - 1)]
    _check_policy([p.cpu().numpy() for p in ro.params], seed, prev, A, LP, 0, N)
    kls, worst, mean_abs = _check_fp32(actor, prev, A, LP, seed, 0, N)
    print("C5 65536 x %d: KL(kernel || fp32) per tick mean %.2e max %.2e, |d logp| max %.3e mean %.2e" % (
        T, np.mean(kls), np.max(np.abs(kls)), worst, mean_abs))
    assert abs(np.mean(kls)) < FP32_KL


def test_fused_policy_without_outputs_and_bad_args():
    """actions/logp outputs are optional; frame_delay > 0 and a wrong actor shape are refused."""
    import torch
    from footsies_gym_amd._lib import FootsiesError
    from footsies_gym_amd.rollout import FusedPolicyRollout, make_actor
    from footsies_gym_amd.simulator import FootsiesSim
    actor = make_actor(device=torch.device("cuda", 0), seed=1)
    a = FootsiesSim(256, p2_mode="bot", seed=4)
    b = FootsiesSim(256, p2_mode="bot", seed=4)
    FusedPolicyRollout(a, actor, seed=3).rollout(30, actions=False, logp=False)
    FusedPolicyRollout(b, actor, seed=3).rollout(30)
    torch.cuda.synchronize()
    for k, v in a.outputs_numpy().items():
        assert np.array_equal(v, b.outputs_numpy()[k]), k
    d = FootsiesSim(8, p2_mode="bot", frame_delay=2)
    with pytest.raises(FootsiesError):
        FusedPolicyRollout(d, actor).rollout(4)
    with pytest.raises(ValueError):
        FusedPolicyRollout(a, make_actor(hidden=32, device=torch.device("cuda", 0)))


@pytest.mark.parametrize("N,horizon,iters,old,learner", [(2048, 32, 3, "behaviour", "hip"),
                                                         (2048, 32, 2, "fp32", "hip"),
                                                         (2048, 32, 2, "behaviour", "torch"),
                                                         (65536, 16, 2, "behaviour", "hip"),
                                                         (2048, 32, 3, "behaviour", "hip_split_bf16")])
def test_ppo_iterations_learn_and_refresh_the_kernel_actor(N, horizon, iters, old, learner):
    """PPOTrainer: fused rollouts + fused-kernel (or torch autograd) updates; losses finite, weights move, and the
    kernel samples from the refreshed weights (the same seed then draws different actions).
    Every iteration reports how far the bf16 behaviour actor is from the fp32 one it trains."""
    import torch
    from footsies_gym_amd.ppo import PPOTrainer
    from footsies_gym_amd.simulator import FootsiesSim
    sim = FootsiesSim(N, p2_mode="bot", seed=5)
    learner, prec = ("hip", "split_bf16") if learner == "hip_split_bf16" else (learner, "fp32")
    tr = PPOTrainer(sim, horizon=horizon, epochs=2, minibatches=4, lr=1e-2, seed=3, old_logp=old, learner=learner,
                    learner_precision=prec)
    w0 = [p.detach().clone() for p in tr.actor.parameters()]
    k0 = [p.clone() for p in tr.rollout.params]
    rate = tr.train(iters)
    assert rate > 0
    for v in tr.stats.values():
        assert bool(torch.isfinite(v))
    kl, gap = float(tr.stats["kl_behaviour_fp32"]), float(tr.stats["logp_abs_diff"])
    print("PPO N=%d old=%s: KL(bf16 || fp32) %.2e, mean |d logp| %.2e" % (N, old, kl, gap))
    assert abs(kl) < 1e-3 and gap < 0.02
    assert any(not torch.equal(a, b) for a, b in zip(w0, tr.actor.parameters()))
    for a, b in zip(tr.rollout.params, tr.actor.parameters()):
        assert torch.equal(a, b.detach())
    assert any(not torch.equal(a, b) for a, b in zip(k0, tr.rollout.params))
    assert sim.steps_taken == iters * horizon


@pytest.mark.parametrize("precision", ["split_bf16", "fp32"])
def test_ppo_critic_values_do_not_depend_on_old_logp(precision):
    """GAE's baseline (the critic values) comes from the learner's own precision whatever
    old_logp is.  Two trainers from the same seed, one per old_logp mode, prepare the same rollout:
    the advantages and returns (rows[:, 10:12]) agree bit for bit, the old log-prob column is the
    behaviour log-prob in one and the fp32 recomputation in the other."""
    import torch
    from footsies_gym_amd.ppo import PPOTrainer
    from footsies_gym_amd.simulator import FootsiesSim
    got = {}
    for old in ("behaviour", "fp32"):
        sim = FootsiesSim(2048, p2_mode="bot", seed=5)
        tr = PPOTrainer(sim, horizon=16, seed=3, old_logp=old, learner_precision=precision)
        rows, gap = tr.prepare(*tr.collect())
        torch.cuda.synchronize()
        got[old] = (rows.clone(), tr.logp.reshape(-1).clone())
        sim.close()
    (rb, behav), (rf, behav2) = got["behaviour"], got["fp32"]
    assert torch.equal(behav, behav2)  # the same rollout in both
    assert torch.equal(rb[:, :9], rf[:, :9]) and torch.equal(rb[:, 10:12], rf[:, 10:12])
    assert torch.equal(rb[:, 9], behav) and not torch.equal(rf[:, 9], behav)
