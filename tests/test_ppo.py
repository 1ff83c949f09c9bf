"""The PPO learner's host logic on CPU: GAE against a plain loop."""
import numpy as np


def test_gae_matches_reference_loop():
    import torch
    from footsies_gym_amd.ppo import gae
    rng = np.random.default_rng(0)
    T, N, gamma, lam = 17, 5, 0.97, 0.9
    r = rng.standard_normal((T, N)).astype(np.float32)
    v = rng.standard_normal((T + 1, N)).astype(np.float32)
    d = (rng.random((T, N)) < 0.2).astype(np.float32)
    adv, ret = gae(torch.from_numpy(r), torch.from_numpy(v), torch.from_numpy(d), gamma, lam)
    want = np.zeros((T, N))
    for n in range(N):
        g = 0.0
        for t in reversed(range(T)):
            nxt = 0.0 if d[t, n] else v[t + 1, n]
            delta = r[t, n] + gamma * nxt - v[t, n]
            g = delta + (0.0 if d[t, n] else gamma * lam * g)
            want[t, n] = g
    assert np.allclose(adv.numpy(), want, atol=1e-5)
    assert np.allclose(ret.numpy(), want + v[:-1], atol=1e-5)


def test_skinny_linear_matches_autograd():
    """The learner's Linear layers (chunked weight-gradient GEMMs) give torch's outputs and, up
    to fp32 summation order, its gradients -- over a row count that leaves a ragged chunk."""
    import torch
    from footsies_gym_amd.ppo import _WGRAD_CHUNK, make_critic, mlp
    from footsies_gym_amd.rollout import make_actor
    torch.manual_seed(0)
    for net in (make_actor(), make_critic()):
        x = torch.randn(2 * _WGRAD_CHUNK + 123, 8)
        y = net(x)
        g = torch.randn_like(y)
        y.backward(g)
        want = [p.grad.clone() for p in net.parameters()]
        for p in net.parameters():
            p.grad = None
        y2 = mlp(net, x)
        y2.backward(g)
        assert torch.equal(y, y2)
        for w, p in zip(want, net.parameters()):
            assert torch.allclose(p.grad, w, rtol=1e-5, atol=1e-4 * float(w.abs().max()))
