"""Host restatement of the in-kernel actor of fs_step_n_policy (footsies_gym_amd/csrc/fs_policy.h),
the checker for its GPU tests.  This is the framework's own C5 actor, not reference code: the
Unity game has no learned actor, so its parity bar is the simulation (bit-exact, by replaying the
sampled actions through the oracle) plus this model of the MLP within a bf16 tolerance.

Numerics restated: inputs and (folded) weights rounded to bf16 (round-to-nearest-even), biases as
bf16 hi + lo pairs, products summed exactly (float64 here; f32 accumulation in the MFMA), the
hidden values r = 1 / (1 + e^(2z)) (tanh z = 1 - 2 r) rounded to bf16 between layers, logits in
f32, then softmax and the inverse-CDF draw with the counter-based uniform `policy_uniform`."""
import numpy as np

C1 = np.uint64(0x9E3779B97F4A7C15)
C2 = np.uint64(0xD1B54A32D192ED03)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)


def bf16(x):
    """float32 -> bf16 (RNE) -> float32."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = (u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) & np.uint64(0xFFFF0000)
    return u.astype(np.uint32).view(np.float32)


def policy_uniform(seed, env, t):
    """fs_policy.h policy_uniform: 24 bits of splitmix64(seed ^ env*C1 ^ t*C2) as a float in [0, 1)."""
    env = np.asarray(env, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = np.uint64(seed) ^ (env * C1) ^ (np.uint64(t) * C2)
        x = x + C1
        x = (x ^ (x >> np.uint64(30))) * M1
        x = (x ^ (x >> np.uint64(27))) * M2
    x = x ^ (x >> np.uint64(31))
    return (x >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def features(out):
    """[N, 8] f32 of one step's outputs (guard, move, move_frame, position: [N, 2] each), ordered
    g1, g2, m1, m2, mf1, mf2, x1, x2 and scaled by the f32 reciprocals the kernel multiplies by."""
    g = np.asarray(out["guard"]).astype(np.float32) * (np.float32(1.0) / np.float32(3.0))
    m = np.asarray(out["move"]).astype(np.float32) * (np.float32(1.0) / np.float32(16.0))
    mf = np.asarray(out["move_frame"], dtype=np.float32) * (np.float32(1.0) / np.float32(55.0))
    x = np.asarray(out["position"], dtype=np.float32) * (np.float32(1.0) / np.float32(4.6))
    return np.concatenate([g, m, mf, x], axis=1).astype(np.float32)


C_TANH = np.float32(2.8853900817779268)  # fs_policy.h kTanhScale = 2 log2(e)


def _bias_pair(b):
    """f32 bias -> its bf16 hi + lo pair (two k slots of the kernel's bias MFMA), summed exactly."""
    b = np.asarray(b, dtype=np.float32)
    hi = bf16(b)
    return hi.astype(np.float64) + bf16(b - hi).astype(np.float64)


def _r(d):
    """r = 1 / (1 + 2^d) in f32, rounded to bf16 (tanh = 1 - 2 r of the unscaled pre-activation)."""
    d = np.asarray(d, dtype=np.float32)
    with np.errstate(over="ignore"):
        return bf16(np.float32(1.0) / (np.float32(1.0) + np.exp2(d)))


def logits(params, feats):
    """params: the six fp32 arrays (w1, b1, w2, b2, w3, b3) in nn.Linear layouts.  Mirrors the
    kernel's folded form: layer 1 pre-scaled by c = 2 log2(e); layers 2 and 3 take r with weights
    -2 W (layer 2 also scaled by c) and biases b + sum_k W[., k]; products summed exactly."""
    w1, b1, w2, b2, w3, b3 = [np.asarray(p, dtype=np.float32) for p in params]
    a1 = bf16(C_TANH * w1).astype(np.float64)
    a2 = bf16(np.float32(-2.0) * C_TANH * w2).astype(np.float64)
    a3 = bf16(np.float32(-2.0) * w3).astype(np.float64)
    c2 = _bias_pair(C_TANH * (b2 + w2.astype(np.float64).sum(axis=1).astype(np.float32)))
    c3 = _bias_pair(b3 + w3.astype(np.float64).sum(axis=1).astype(np.float32))
    r1 = _r(bf16(feats).astype(np.float64) @ a1.T + _bias_pair(C_TANH * b1))
    r2 = _r(r1.astype(np.float64) @ a2.T + c2)
    return (r2.astype(np.float64) @ a3.T + c3).astype(np.float32)


def sample(lg, u):
    """Inverse-CDF draw per row of logits `lg` [N, 8] with uniforms `u` [N]; returns
    (action, logp, margin): margin is how far (in probability) u sits from the nearest CDF
    boundary, below which rounding may legitimately pick the neighbouring action."""
    z = lg.astype(np.float64) - lg.max(axis=1, keepdims=True)
    p = np.exp(z)
    p /= p.sum(axis=1, keepdims=True)
    cdf = np.cumsum(p, axis=1)
    act = np.minimum((u[:, None] >= cdf).sum(axis=1), 7)
    margin = np.abs(cdf[:, :7] - u[:, None].astype(np.float64)).min(axis=1)
    logp = np.log(p[np.arange(len(act)), act])
    return act.astype(np.uint8), logp.astype(np.float32), margin
