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
