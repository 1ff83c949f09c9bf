"""fs_step_n_policy: the C5 actor inside the fused tick loop (csrc/fs_policy.h).

Two bars.  The simulation stays bit-exact: the actions the kernel sampled, replayed through
the oracle, give the same per-tick trajectory and final state.  The actor matches its host
restatement (tests/policy_ref.py): the same action wherever the uniform is not within
rounding distance of a CDF boundary, and log-probabilities within 0.05 (bf16 inputs, weights
and hidden activations; f32 accumulation)."""
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


def test_ppo_iterations_learn_and_refresh_the_kernel_actor():
    """PPOTrainer: fused rollouts + torch updates; losses finite, weights move, and the
    kernel samples from the refreshed weights (the same seed then draws different actions)."""
    import torch
    from footsies_gym_amd.ppo import PPOTrainer
    from footsies_gym_amd.simulator import FootsiesSim
    sim = FootsiesSim(2048, p2_mode="bot", seed=5)
    tr = PPOTrainer(sim, horizon=32, epochs=2, minibatches=4, lr=1e-2, seed=3)
    w0 = [p.detach().clone() for p in tr.actor.parameters()]
    k0 = [p.clone() for p in tr.rollout.params]
    rate = tr.train(3)
    assert rate > 0
    for v in tr.stats.values():
        assert bool(torch.isfinite(v))
    assert any(not torch.equal(a, b) for a, b in zip(w0, tr.actor.parameters()))
    for a, b in zip(tr.rollout.params, tr.actor.parameters()):
        assert torch.equal(a, b.detach())
    assert any(not torch.equal(a, b) for a, b in zip(k0, tr.rollout.params))
    assert sim.steps_taken == 3 * 32
