"""The host restatement of the fused actor (tests/policy_ref.py) on CPU: its bf16 rounding is
torch's, its MLP is make_actor's forward within bf16 error, its uniforms are in [0, 1)."""
import numpy as np

from tests import policy_ref


def test_bf16_rounding_matches_torch():
    import torch
    x = np.random.default_rng(0).standard_normal(100000).astype(np.float32) * 10
    x[:4] = [0.0, -0.0, 1.0 + 2.0**-8, 1.0 + 3 * 2.0**-8]  # exact ties round to even
    want = torch.from_numpy(x).to(torch.bfloat16).float().numpy()
    assert np.array_equal(policy_ref.bf16(x).view(np.uint32), want.view(np.uint32))


def test_logits_track_the_fp32_actor():
    import torch
    from footsies_gym_amd.rollout import make_actor
    actor = make_actor(seed=2)
    params = [p.detach().numpy() for p in actor.parameters()]
    rng = np.random.default_rng(1)
    out = {"guard": rng.integers(0, 4, (512, 2)), "move": rng.integers(0, 17, (512, 2)),
           "move_frame": rng.integers(0, 56, (512, 2)).astype(np.float32),
           "position": rng.uniform(-4.6, 4.6, (512, 2)).astype(np.float32)}
    f = policy_ref.features(out)
    with torch.no_grad():
        want = actor(torch.from_numpy(f)).numpy()
    got = policy_ref.logits(params, f)
    assert np.abs(got - want).max() < 0.1


def test_uniform_range_and_sampling():
    u = policy_ref.policy_uniform(0xC0FFEE, np.arange(100000), 7)
    assert u.min() >= 0.0 and u.max() < 1.0 and abs(u.mean() - 0.5) < 0.01
    assert not np.array_equal(u, policy_ref.policy_uniform(0xC0FFEE, np.arange(100000), 8))
    lg = np.zeros((100000, 8), dtype=np.float32)
    act, logp, _ = policy_ref.sample(lg, u)
    assert np.bincount(act, minlength=8).min() > 11000
    assert np.allclose(logp, np.log(1 / 8))
